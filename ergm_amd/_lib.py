"""ctypes binding of libergm_hip.so (the C-ABI declared in include/ergm_hip.h).

The library is loaded from the package directory (built in-tree by ``ergm_amd/build.py``).  There
is no fallback: if the library is missing or fails to load, every op raises — the product path never
silently runs on CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libergm_hip.so")

ABI_VERSION = 11  # ERGM_ABI_VERSION of include/ergm_hip.h this binding matches
ERGM_OK, ERGM_EINVAL, ERGM_EUNSUPPORTED, ERGM_EHIP = 0, -1, -2, -3
F32, BF16 = 0, 1
MK, KM = 0, 1
NK, KN = 0, 1
EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RESID, EPI_GELU_BWD, EPI_ACCUM = range(6)
LAYER_TENSORS = ["ln_1.weight", "ln_1.bias", "attn.c_attn.weight", "attn.c_attn.bias", "attn.c_proj.weight",
                 "attn.c_proj.bias", "ln_cross_attn.weight", "ln_cross_attn.bias",
                 "crossattention.q_attn.weight", "crossattention.q_attn.bias", "crossattention.c_proj.weight",
                 "crossattention.c_proj.bias", "ln_2.weight", "ln_2.bias", "mlp.c_fc.weight", "mlp.c_fc.bias",
                 "mlp.c_proj.weight", "mlp.c_proj.bias"]  # order of ergm_layer_tensor


class Dropout(C.Structure):
    """ergm_dropout: one dropout site of one forward (ergm_hip.h)."""
    _fields_ = [("seed", C.c_uint64), ("offset", C.c_uint32), ("site", C.c_uint32), ("p", C.c_float),
                ("row0", C.c_int64)]


class GemmDesc(C.Structure):
    _fields_ = [("M", C.c_int), ("N", C.c_int), ("K", C.c_int), ("lda", C.c_int), ("ldb", C.c_int),
                ("ldc", C.c_int), ("a_layout", C.c_int), ("b_layout", C.c_int), ("c_dtype", C.c_int),
                ("epilogue", C.c_int), ("alpha", C.c_float), ("bias", C.c_void_p), ("aux", C.c_void_p),
                ("ld_aux", C.c_int), ("aux_out", C.c_void_p), ("ld_aux_out", C.c_int), ("split_k", C.c_int),
                ("alpha_dev", C.c_void_p), ("dropout", C.POINTER(Dropout)), ("bias_grad", C.c_void_p)]


class AdamWDesc(C.Structure):
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p),
                ("param_bf16", C.c_void_p), ("ranges", C.POINTER(C.c_int64)), ("n_ranges", C.c_int),
                ("wte_begin", C.c_int64), ("lr", C.c_double), ("beta1", C.c_double), ("beta2", C.c_double),
                ("weight_decay", C.c_double), ("eps", C.c_float), ("step_size", C.c_float), ("bc2_sqrt", C.c_float),
                ("max_blocks", C.c_int), ("defer", C.c_int)]


class ModelDims(C.Structure):
    _fields_ = [("vocab", C.c_int), ("vocab_pad", C.c_int), ("n_embd", C.c_int), ("n_layer", C.c_int),
                ("n_head", C.c_int), ("n_inner", C.c_int), ("n_positions", C.c_int), ("batch", C.c_int),
                ("seq", C.c_int), ("eps", C.c_float), ("has_features", C.c_int), ("ld_vis", C.c_int),
                ("feat_dim", C.c_int), ("fp8", C.c_int)]


class ModelParams(C.Structure):
    _fields_ = [("wte", C.c_void_p), ("wte_b", C.c_void_p), ("wpe", C.c_void_p), ("ln_f_w", C.c_void_p),
                ("ln_f_b", C.c_void_p), ("emo_w", C.c_void_p), ("capkv_w_b", C.c_void_p), ("capkv_b", C.c_void_p),
                ("layer_f32", C.c_void_p), ("layer_b16", C.c_void_p), ("layer_stride", C.c_int64),
                ("layer_off", C.c_int64 * 18),
                ("g_wte", C.c_void_p), ("g_wpe", C.c_void_p), ("g_ln_f_w", C.c_void_p), ("g_ln_f_b", C.c_void_p),
                ("g_emo_w", C.c_void_p), ("g_capkv_w", C.c_void_p), ("g_capkv_b", C.c_void_p),
                ("g_layer", C.c_void_p),
                ("vproj_w_b", C.c_void_p), ("vproj_b", C.c_void_p), ("aproj_w_b", C.c_void_p),
                ("aproj_b", C.c_void_p), ("g_vproj_w", C.c_void_p), ("g_vproj_b", C.c_void_p),
                ("g_aproj_w", C.c_void_p), ("g_aproj_b", C.c_void_p), ("capkv_w", C.c_void_p)]


vp, i32, i64, f32, f64, sz = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_double, C.c_size_t
_SIGS = {
    "ergm_version": (i32, []),
    "ergm_last_error": (i32, [C.c_char_p, sz]),
    "ergm_gemm_tune": (i32, [i32, i32]),
    "ergm_gemm_set_override": (i32, [i32, i32, i32, i32, i32, i32, i32]),
    "ergm_gemm_trace": (i32, [i32, vp, i32]),
    "ergm_gemm_workspace_size": (sz, [C.POINTER(GemmDesc)]),
    "ergm_gemm": (i32, [C.POINTER(GemmDesc), vp, vp, vp, vp, sz, vp]),
    "ergm_gemm_f8": (i32, [C.POINTER(GemmDesc), vp, vp, vp, vp, vp, vp]),
    "ergm_gemm_f8_tune": (i32, [i32]),
    "ergm_gemm_f8_set_override": (i32, [i32, i32, i32, i32]),
    "ergm_quant_rows_fp8": (i32, [vp, i32, i32, i32, i32, vp, i32, vp, vp]),
    "ergm_quant_weight_fp8": (i32, [vp, i32, i32, i32, i32, vp, i32, vp, vp, vp]),
    "ergm_gemm_mx": (i32, [C.POINTER(GemmDesc), vp, vp, i32, vp, vp, i32, vp, vp, vp, i32, i32, vp]),
    "ergm_quant_rows_mx": (i32, [vp, i32, i32, i32, i32, vp, i32, vp, i32, vp]),
    "ergm_quant_weight_mx": (i32, [vp, i32, i32, i32, vp, i32, vp, i32, vp, i32, vp, i32, vp]),
    "ergm_attn_fwd": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    "ergm_attn_tune": (i32, [i32]),
    "ergm_attn_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp] + [i32] * 13 + [vp, vp, vp]),
    "ergm_layernorm_fwd": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, f32, vp]),
    "ergm_layernorm_bwd_workspace_size": (sz, [i32, i32]),
    "ergm_layernorm_bwd": (i32, [vp] * 10 + [sz, i32, i32, vp, vp]),
    "ergm_dropout_mask": (i32, [vp, i32, i32, vp, vp]),
    "ergm_dropout_apply": (i32, [vp, vp, i32, i32, i32, vp]),
    "ergm_colsum_workspace_size": (sz, [i32, i32]),
    "ergm_colsum": (i32, [vp, i32, i32, i32, i32, vp, i32, vp, sz, vp]),
    "ergm_embed_fwd": (i32, [vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, i32, i32, vp, vp]),
    "ergm_feat_pool": (i32, [vp, i32, i32, i32, i32, C.c_long, C.c_long, vp, vp, i32, vp]),
    "ergm_embed_bwd_workspace_size": (sz, [i32]),
    "ergm_embed_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, sz, i32, i32, i32, i32, vp]),
    "ergm_count_valid": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "ergm_xent_fwd_bwd": (i32, [vp, i32, vp, vp, vp, vp, i32, i32, i32, f32, vp]),
    "ergm_emotion_head": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp, vp, vp]),
    "ergm_loss_finalize": (i32, [vp, i32, vp, vp, vp, vp, vp]),
    "ergm_adamw_step": (i32, [vp, vp, vp, vp, vp, sz, f64, f64, f64, f32, f64, f32, f32, i32, vp]),
    "ergm_adamw_rows": (i32, [vp, vp, vp, vp, vp, i32, i32, vp, i32, f64, f64, f64, f32, f64, f32, f32, i32, vp]),
    "ergm_cast_bf16": (i32, [vp, vp, sz, vp]),
    "ergm_axpy": (i32, [vp, vp, sz, f32, vp]),
    "ergm_chunk_sum_bf16": (i32, [vp, i32, sz, vp, vp]),
    "ergm_chunk_sum_bf16_f32": (i32, [vp, i32, sz, sz, vp, vp]),
    "ergm_cast_f32": (i32, [vp, vp, sz, vp]),
    "ergm_dp_pack_bf16": (i32, [vp, sz, vp, sz, vp]),
    "ergm_dp_sum_adamw": (i32, [vp, i32, sz, sz, vp, vp, vp, vp, vp, f64, f64, f64, f32, f64, f32, f32, i32, vp]),
    "ergm_model_workspace_size": (sz, [C.POINTER(ModelDims)]),
    "ergm_model_create": (i32, [C.POINTER(ModelDims), C.POINTER(ModelParams), vp, sz, C.POINTER(vp)]),
    "ergm_model_destroy": (i32, [vp]),
    "ergm_model_set_probe": (i32, [vp, i32, vp, vp]),
    "ergm_model_set_optimizer": (i32, [vp, vp]),
    "ergm_model_optimizer_join": (i32, [vp, vp]),
    "ergm_model_set_probe_list": (i32, [vp, i32, vp, vp, vp, i32]),
    "ergm_model_probe_count": (i32, [vp]),
    "ergm_model_set_row_flags": (i32, [vp, vp, i32]),
    "ergm_model_set_lookup_compact": (i32, [vp, vp, vp]),
    "ergm_rows_scan": (i32, [vp, i32, vp, vp, vp]),
    "ergm_rows_compact": (i32, [vp, vp, i32, i32, vp, vp, i32, vp]),
    "ergm_model_set_inputs": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "ergm_model_set_dropout": (i32, [vp, f32, f32, f32, C.c_uint64, C.c_uint32, i32]),
    "ergm_model_forward": (i32, [vp, vp, vp, vp, i32, vp]),
    "ergm_model_backward_head": (i32, [vp, vp, vp]),
    "ergm_model_backward_layer": (i32, [vp, i32, vp]),
    "ergm_model_backward_embed": (i32, [vp, vp]),
    "ergm_model_set_side_joins": (i32, [vp, i32]),
    "ergm_model_set_metrics": (i32, [vp, vp, vp]),
    "ergm_model_set_logits_grad": (i32, [vp, vp]),
    "ergm_model_stage_wait": (i32, [vp, i32, vp]),
}
EXPORTED = sorted(_SIGS)

_lib = None
_lock = threading.Lock()


class ErgmError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load (once) and return the library; raises if it is missing.  ERGM_LIB_PATH overrides the path
    (A/B runs of two builds of the same sources)."""
    path = os.environ.get("ERGM_LIB_PATH", path)
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise ErgmError(f"libergm_hip.so not found at {path}: run `python -m ergm_amd.build` "
                                "(the HIP path has no CPU fallback)")
            lib = C.CDLL(path)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            if lib.ergm_version() != ABI_VERSION:
                raise ErgmError(f"{path} has ABI {lib.ergm_version()}, this binding expects {ABI_VERSION}: rebuild "
                                "with `python -m ergm_amd.build`")
            _lib = lib
    return _lib


def last_error() -> str:
    buf = C.create_string_buffer(512)
    load().ergm_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(rc: int, what: str) -> None:
    """Map a C status to the reference's exception types (ValueError for bad arguments)."""
    if rc == ERGM_OK:
        return
    msg = f"{what}: {last_error()}"
    if rc == ERGM_EINVAL:
        raise ValueError(msg)
    if rc == ERGM_EUNSUPPORTED:
        raise NotImplementedError(msg)
    raise ErgmError(msg)


def _hip():
    if HipEvent._hip is None:
        h = C.CDLL("libamdhip64.so")
        h.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
        h.hipEventDestroy.argtypes = [C.c_void_p]
        h.hipEventSynchronize.argtypes = [C.c_void_p]
        h.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        h.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        h.hipStreamWaitEvent.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
        HipEvent._hip = h
    return HipEvent._hip


HIP_EVENT_DISABLE_TIMING = 0x2
HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000  # device-scope release: no L2 writeback at record time


class HipEvent:
    """A raw hipEvent_t (libamdhip64).  Default: a timing event for the executor's in-loop probe;
    ``sync=True``: a device-scope ordering event between two streams of one device (no timing, no
    system-scope fence, so recording it on the critical stream costs no cache writeback)."""
    _hip = None

    def __init__(self, sync: bool = False):
        h = _hip()
        flags = HIP_EVENT_DISABLE_SYSTEM_FENCE | (HIP_EVENT_DISABLE_TIMING if sync else 0)
        self.ev = C.c_void_p()
        if h.hipEventCreateWithFlags(C.byref(self.ev), flags) != 0:
            raise ErgmError("hipEventCreateWithFlags failed")

    def record(self, stream) -> None:
        if _hip().hipEventRecord(self.ev, C.c_void_p(stream)) != 0:
            raise ErgmError("hipEventRecord failed")

    def wait(self, stream) -> None:
        """Make `stream` (a hipStream_t as int) wait for the last record of this event."""
        if _hip().hipStreamWaitEvent(C.c_void_p(stream), self.ev, 0) != 0:
            raise ErgmError("hipStreamWaitEvent failed")

    def elapsed_ms(self, end: "HipEvent") -> float:
        h = _hip()
        if h.hipEventSynchronize(end.ev) != 0:
            raise ErgmError("hipEventSynchronize failed")
        ms = C.c_float()
        rc = h.hipEventElapsedTime(C.byref(ms), self.ev, end.ev)
        if rc != 0:
            raise ErgmError(f"hipEventElapsedTime failed ({rc})")
        return ms.value

    def __del__(self):
        try:
            if self.ev and HipEvent._hip is not None:
                HipEvent._hip.hipEventDestroy(self.ev)
        except Exception:
            pass


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)
