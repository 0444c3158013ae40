"""CPU oracle for the ERGM hot path (test infrastructure only; see gpt2_oracle.py)."""
