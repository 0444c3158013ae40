"""ergm_amd: MI355X-native fused GPT-2 (ERGM) training step."""
