"""ctypes binding of the C ABI in include/vsiq.h (the drop-in boundary).

The library is loaded AFTER torch so that its NEEDED `libamdhip64.so.7` resolves
to the HIP runtime torch already mapped (same soname): one HIP runtime, one
context, and torch's stream handles are valid inside the kernels' launches.

Fails loudly: there is no CPU fallback anywhere in vsiquantization_amd.  A
missing library, a CPU tensor, or a non-zero return code raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from . import _build

_LIB = None
_LOCK = threading.Lock()

c_p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_d = ctypes.c_double

ABI_VERSION = 11
COUNTER_WORDS = 64   # VSIQ_COUNTER_WORDS
COUNTER_GRID_ERRORS = 35   # VSIQ_COUNTER_GRID_ERRORS (K10's barrier-timeout count)

# record layouts (include/vsiq.h)
ST_MIN, ST_MAX, ST_NAN, ST_SUMABS, ST_SUM, ST_SUMSQ, ST_N, ST_MEANABS, ST_MEAN, ST_STD = range(10)
ST_LEN = 10
PART_LEN = 8   # VSIQ_PART_LEN: doubles per K2p partial record
PART_MAX_RECORDS = 4096   # VSIQ_PART_MAX_RECORDS
QP_SCALE, QP_ZP, QP_MIN, QP_MAX = range(4)
QP_LEN = 4
TUNE_NONTEMPORAL, TUNE_STORE_DEFER = 2, 6
TUNE_OBS_KERNEL, TUNE_LSQ_GROUPS, TUNE_PC_PACKED = 7, 9, 10
TUNE_STORE_GATE = 11
TUNE_GATE_AUTOTUNE = 12
TUNE_XCD_ORDER = 13
TUNE_K2O_FORM, TUNE_K2O_GROUPS, TUNE_K2O_BLOCK = 14, 15, 17
REMOVED_TUNE_KEYS = (1, 5, 8, 16)   # ABI 10: K3 rows / workgroup size, K2 grid, K2 cached-load threshold
ACT_NONE, ACT_RELU, ACT_SILU = 0, 1, 2
ACT_CODES = {None: ACT_NONE, "none": ACT_NONE, "relu": ACT_RELU, "silu": ACT_SILU}

# SiLU bit for bit as torch's CPU kernel on this host (include/vsiq.h VSIQ_ACT_SILU_REF):
# which elements torch computes with glibc's scalar expf instead of the vectorized Sleef
# exp depends on the vector width of torch's CPU kernels and on its thread count.
_SILU_W = {"AVX512": 32, "AVX2": 16}
_SILU_PIN = []   # set_silu_reference(): (W, threads) instead of this host's


def set_silu_reference(width=None, threads=None):
    """Pin the reference CPU layout SiLU is reproduced for: ``width`` = 2 x floats per
    vector (32 AVX-512, 16 AVX2, 0 = every element on the vectorized path), ``threads`` =
    torch's CPU thread count.  No arguments: follow this host's torch (the default)."""
    _SILU_PIN.clear()
    if width is not None:
        if width not in (0, 8, 16, 32, 64) or not 0 <= int(threads or 0) < 32768:
            raise ValueError(f"silu reference width {width} / threads {threads}")
        _SILU_PIN.append((int(width), int(threads or 1)))


def silu_reference():
    """(W, threads) of the reference CPU layout act="silu" reproduces."""
    if _SILU_PIN:
        return _SILU_PIN[0]
    return _SILU_W.get(torch.backends.cpu.get_cpu_capability(), 16), torch.get_num_threads()


# mean|x| / mean x of an observer call as torch's CPU kernel sums them (K11,
# csrc/k_mean.hip): off by default (the stats are the correctly rounded fp32 means of
# an f64 sum, within one fp32 ulp of torch's; K11 costs one extra read per call).  On:
# (vec, threads) of the reference host -- vec 8 is the Vectorized<float> this torch
# build's sum kernel uses on AVX2 and AVX-512 hosts alike (tests/test_mean_oracle.py).
_MEAN_REF = []


def set_mean_reference(threads=None, vec: int = 8):
    """Record mean|x| / mean x bit for bit as torch's CPU torch.mean on a host with
    ``threads`` CPU threads (None: this process's torch.get_num_threads()); the reference
    records those values (quantization_manager.py:66-67) and builds the learnable scale
    from them (qm.py:112).  Costs one extra read of each observed tensor."""
    t = torch.get_num_threads() if threads is None else int(threads)
    if vec not in (8, 16) or not 1 <= t <= 4096:
        raise ValueError(f"mean reference vec {vec} / threads {t}")
    _MEAN_REF[:] = [(int(vec), t)]


def clear_mean_reference():
    """Back to the default statistics (no extra pass)."""
    _MEAN_REF.clear()


def mean_reference():
    """(vec, threads) of the reference layout mean|x| / mean x follow, or None (off)."""
    return _MEAN_REF[0] if _MEAN_REF else None


def _mean_reference_from_env():
    v = os.environ.get("VSIQ_MEAN_REFERENCE", "").strip()
    if not v or v == "0":
        return
    if v == "host":
        set_mean_reference()
    elif "," in v:
        a, b = v.split(",", 1)
        set_mean_reference(int(b), int(a))
    else:
        set_mean_reference(int(v))


_mean_reference_from_env()


class SiluAct(str):
    """act="silu" bound to one reference CPU layout (W, threads) instead of the process's
    (silu_reference()): a QuantizationManager passes its recorded layout this way, so a
    layer keeps the SiLU bits its qparams were observed / learned with.  Compares and
    hashes as "silu"."""

    def __new__(cls, width, threads):
        s = super().__new__(cls, "silu")
        s.layout = (int(width), int(threads))
        return s

    def __reduce__(self):
        return (SiluAct, self.layout)


def act_code(act) -> int:
    """None / "relu" / "silu" (or the VSIQ_ACT_* integer) -> the C ABI act argument
    (SiLU carries the reference CPU layout, VSIQ_ACT_SILU_REF)."""
    if isinstance(act, SiluAct):
        w, t = act.layout
        return ACT_SILU | (w << 8) | (min(max(t, 0), 32767) << 16)
    if isinstance(act, int) and act in (ACT_NONE, ACT_RELU, ACT_SILU):
        code = act
    else:
        try:
            code = ACT_CODES[act]
        except KeyError:
            raise ValueError(f"unsupported fused activation {act!r} (None, 'relu' or 'silu')") from None
    if code == ACT_SILU:
        w, t = silu_reference()
        return ACT_SILU | (w << 8) | (min(max(t, 0), 32767) << 16)
    return code


def act_kind(code: int) -> int:
    """The activation of a C ABI act argument (low byte)."""
    return code & 0xff

_SIGS = {
    "vsiq_abi_version": ([], c_int),
    "vsiq_error_string": ([c_int], ctypes.c_char_p),
    "vsiq_workspace_doubles": ([c_i64], c_i64),
    "vsiq_mask_words": ([c_i64, c_i64], c_i64),
    "vsiq_set_tuning": ([c_int, c_int], c_int),
    "vsiq_gate_tuning_pending": ([], c_int),
    "vsiq_gate_report": ([ctypes.c_char_p, c_i64], c_i64),
    "vsiq_gate_reset": ([], c_int),
    "vsiq_gate_retune": ([], c_int),
    "vsiq_gate_export": ([ctypes.c_char_p, c_i64], c_i64),
    "vsiq_gate_import": ([ctypes.c_char_p], c_int),
    "vsiq_gate_freeze": ([c_int], c_int),
    "vsiq_trace_marker": ([c_int, c_p], c_int),
    "vsiq_torch_mean_ws_bytes": ([c_i64, c_int, c_int], c_i64),
    "vsiq_torch_mean_f32": ([c_p, c_i64, c_int, c_int, c_int, c_p, c_p, c_p, c_i64, c_p], c_int),
    "vsiq_host_torch_mean_f32": ([c_p, c_i64, c_int, c_int, c_int, c_p], c_int),
    "vsiq_selftest_div": ([c_p, c_int, c_p, c_p], c_int),
    "vsiq_selftest_fq": ([c_int, c_p, c_p, c_int, ctypes.c_float, ctypes.c_float, c_p, c_p], c_int),
    "vsiq_fq_fwd_f32": ([c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_d, c_p, c_d, c_int, c_int, c_int, c_int, c_p],
                        c_int),
    "vsiq_observe_f32": ([c_p, c_i64, c_p, c_p, c_p, c_int, c_d, c_d, c_p, c_i64, c_p, c_p], c_int),
    "vsiq_observe_finalize": ([c_p, c_p, c_p, c_int, c_d, c_d, c_p], c_int),
    "vsiq_observe_finalize_ranks": ([c_p, c_int, c_p, c_p, c_p, c_int, c_d, c_d, c_p], c_int),
    "vsiq_act_fq_fwd_ranks_f32": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_p, c_int, c_p, c_p, c_p, c_int, c_d, c_d,
                                   c_int, c_int, c_p], c_int),
    "vsiq_pc_observe_fq_f32": ([c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_int, c_int,
                                c_int, c_d, c_d, c_p], c_int),
    "vsiq_pc_fq_fwd_f32": ([c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_int, c_int, c_int, c_p], c_int),
    "vsiq_ste_bwd_f32": ([c_p, c_p, c_p, c_i64, c_p, c_i64, c_d, c_p], c_int),
    "vsiq_lsq_bwd_f32": ([c_p, c_p, c_p, c_i64, c_p, c_d, c_p, c_d, c_int, c_int, c_int, c_d, c_p, c_p,
                          c_i64, c_p, c_p], c_int),
    "vsiq_pcm_fq_fwd_f32": ([c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_int, c_int, c_int, c_p],
                            c_int),
    "vsiq_pcm_workspace_doubles": ([c_i64, c_i64], c_i64),
    "vsiq_pcm_lsq_bwd_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_int, c_int, c_int, c_d, c_p,
                              c_p, c_p, c_i64, c_p], c_int),
    "vsiq_pcm_lsq_bwd_arrive_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_int, c_int, c_int, c_d, c_p,
                                     c_p, c_p, c_i64, c_p, c_i64, c_p], c_int),
    "vsiq_bn_fold_f32": ([c_p, c_p, c_p, c_p, c_p, c_p, ctypes.c_float, c_p, c_p, c_i64, c_i64, c_p], c_int),
    "vsiq_act_fq_fwd_f32": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_p, c_p, c_d, c_p, c_d, c_int, c_int,
                             c_int, c_int, c_p], c_int),
    "vsiq_act_observe_f32": ([c_p, c_i64, c_int, c_p, c_p, c_p, c_int, c_d, c_d, c_p, c_i64, c_p, c_p],
                             c_int),
    "vsiq_observe_part_records": ([c_i64], c_i64),
    "vsiq_observe_part_out_records": ([c_i64], c_i64),
    "vsiq_act_observe_part_f32": ([c_p, c_i64, c_int, c_p, c_i64, c_p], c_int),
    "vsiq_act_observe_part_multi_f32": ([c_p, c_int, c_int, c_p], c_int),
    "vsiq_act_observe_part_out_f32": ([c_p, c_p, c_i64, c_int, c_p, c_i64, c_p], c_int),
    "vsiq_lsq_part_records": ([c_i64], c_i64),
    "vsiq_act_lsq_bwd_part_f32": ([c_p, c_p, c_p, c_i64, c_int, c_p, c_d, c_p, c_d, c_int, c_int, c_int, c_p, c_i64,
                                   c_p], c_int),
    "vsiq_lsq_fold_multi": ([c_p, c_int, c_p], c_int),
    "vsiq_observe_fq_max_elems": ([], c_i64),
    "vsiq_act_observe_fq_f32": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_p, c_p, c_p, c_int, c_d, c_d, c_int, c_int,
                                 c_p], c_int),
    "vsiq_observe_fq_parts_max_elems": ([], c_i64),
    "vsiq_act_observe_fq_parts_f32": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_p, c_p, c_p, c_int, c_d, c_d, c_int,
                                       c_int, c_p, c_i64, c_p], c_int),
    "vsiq_act_observe_fq_grid_f32": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_p, c_p, c_p, c_int, c_d, c_d, c_int,
                                      c_int, c_p, c_i64, c_p, c_p], c_int),
    "vsiq_observe_fold_parts": ([c_p, c_i64, c_i64, c_p, c_p], c_int),
    "vsiq_lsq_multi_workspace_doubles": ([c_p, c_int], c_i64),
    "vsiq_lsq_fwd_multi_f32": ([c_p, c_int, c_p], c_int),
    "vsiq_lsq_bwd_multi_f32": ([c_p, c_int, c_p, c_i64, c_p, c_p], c_int),
    "vsiq_host_observe_f32": ([c_p, c_i64, c_int, c_p, c_p, c_p, c_int, c_d, c_d], c_int),
    "vsiq_host_fq_fwd_f32": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_p, c_d, c_d, c_int, c_int, c_int, c_int], c_int),
    "vsiq_host_ste_bwd_f32": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_d], c_int),
    "vsiq_host_lsq_bwd_f32": ([c_p, c_p, c_p, c_i64, c_int, c_d, c_d, c_int, c_int, c_int, c_d, c_p], c_int),
    "vsiq_host_pc_observe_fq_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_int, c_d, c_d, c_int,
                                     c_int], c_int),
    "vsiq_host_pc_fq_fwd_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_int, c_int, c_int], c_int),
    "vsiq_host_pc_ste_bwd_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_p], c_int),
    "vsiq_host_pcm_fq_fwd_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_int, c_int, c_int], c_int),
    "vsiq_host_pcm_ste_bwd_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p], c_int),
    "vsiq_host_pcm_lsq_bwd_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_int, c_int, c_int, c_d, c_p, c_p],
                                  c_int),
    "vsiq_host_pc_lsq_bwd_f32": ([c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_int, c_int, c_int, c_d, c_p, c_p],
                                 c_int),
    "vsiq_host_threads": ([], c_int),
    "vsiq_host_simd": ([], c_int),
    "vsiq_act_fwd_f32": ([c_p, c_p, c_i64, c_int, c_p], c_int),
    "vsiq_act_bwd_f32": ([c_p, c_p, c_p, c_i64, c_int, c_p], c_int),
    "vsiq_selftest_exp_f32": ([c_p, c_p, c_p, c_i64, c_p], c_int),
    "vsiq_act_ste_bwd_f32": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_p, c_i64, c_d, c_p], c_int),
    "vsiq_act_lsq_bwd_f32": ([c_p, c_p, c_p, c_i64, c_int, c_p, c_d, c_p, c_d, c_int, c_int, c_int, c_d,
                              c_p, c_p, c_i64, c_p, c_p], c_int),
}
EXPORTED = tuple(_SIGS)


class LsqTensor(ctypes.Structure):
    """vsiq_lsq_tensor (include/vsiq.h): one tensor of a multi-tensor learnable launch."""
    _fields_ = [("x", c_p), ("y", c_p), ("g", c_p), ("gx", c_p), ("scale_dev", c_p), ("zp_dev", c_p),
                ("grad_out", c_p), ("n", c_i64), ("scale_host", c_d), ("zp_host", c_d), ("gscale", c_d),
                ("qmin", ctypes.c_int32), ("qmax", ctypes.c_int32), ("zp_learn", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class LsqFold(ctypes.Structure):
    """vsiq_lsq_fold (include/vsiq.h): one call of a deferred scale-gradient fold."""
    _fields_ = [("records", c_p), ("nrec", c_i64), ("zp_dev", c_p), ("zp_host", c_d), ("gscale", c_d),
                ("grad_out", c_p), ("qmin", ctypes.c_int32), ("qmax", ctypes.c_int32), ("zp_learn", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class PartTensor(ctypes.Structure):
    """vsiq_part_tensor (include/vsiq.h): one call of a multi-tensor deferred observer launch."""
    _fields_ = [("c", c_p), ("n", c_i64), ("parts", c_p), ("parts_len", c_i64)]


class VsiqError(RuntimeError):
    pass


def library_path() -> str:
    # VSIQ_LIBRARY: experiments only (tools/exp), e.g. a variant build of the same ABI
    return os.environ.get("VSIQ_LIBRARY") or _build.OUT


def lib():
    """Load (never build) the HIP library; raise if it is absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = library_path()
        if not os.path.exists(path):
            raise VsiqError(
                f"vsiquantization_amd HIP library missing at {path}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        handle = ctypes.CDLL(path)
        for name, (args, res) in _SIGS.items():
            fn = getattr(handle, name)
            fn.argtypes = args
            fn.restype = res
        v = handle.vsiq_abi_version()
        if v != ABI_VERSION:
            raise VsiqError(f"vsiq ABI version {v} != expected {ABI_VERSION}; rebuild the library")
        # VSIQ_GATE_TABLE=<file of gate_save>: start from a saved store-gate table, frozen
        # unless VSIQ_GATE_FREEZE=0 (reproducible kernel timing, no tuner launches)
        table = os.environ.get("VSIQ_GATE_TABLE")
        if table:
            with open(table) as f:
                if handle.vsiq_gate_import(f.read().encode()) < 0:
                    raise VsiqError(f"VSIQ_GATE_TABLE={table}: malformed gate table")
            if os.environ.get("VSIQ_GATE_FREEZE", "1") != "0":
                handle.vsiq_gate_freeze(1)
        _LIB = handle
    return _LIB


_EXT = None


_TORCH_EXT_ON = os.environ.get("VSIQ_TORCH_EXT", "1") != "0"   # read once: every per-call op asks


def torch_ext_enabled() -> bool:
    """VSIQ_TORCH_EXT=0 (in the environment at import) routes the per-call autograd paths
    through the Python autograd.Functions over ctypes instead (same kernels; tests compare
    the two by patching this function)."""
    return _TORCH_EXT_ON


def torch_ext():
    """The C++ autograd nodes (`_vsiq_torch.so`, csrc/torch_ops.cpp); raise if absent."""
    global _EXT
    if _EXT is None:
        lib()   # the HIP library first (ABI check), then the module linked to it
        try:
            from . import _vsiq_torch
        except ImportError as e:
            raise VsiqError(
                f"vsiquantization_amd torch extension _vsiq_torch.so missing or not loadable ({e}); "
                "build it with `python -c 'import __graft_entry__ as g; g.build()'`") from None
        if _vsiq_torch.abi_version() != ABI_VERSION:
            raise VsiqError("_vsiq_torch.so was linked against another vsiq ABI; rebuild")
        _EXT = _vsiq_torch
    return _EXT


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().vsiq_error_string(rc)
        raise VsiqError(f"{what} failed ({rc}): {msg.decode() if msg else '?'}")


# --------------------------------------------------------------------------- tensor helpers
def require_device_f32(x: torch.Tensor, what: str = "x") -> torch.Tensor:
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"{what} must be a torch.Tensor, got {type(x).__name__}")
    if x.device.type != "cuda":
        raise VsiqError(
            f"{what} is on {x.device}: this operation runs on MI355X (HIP) only. CPU float32 "
            "tensors are served by the native host path of the reference's classes "
            "(UniformQuantizer, LSQQuantizer, MinMaxObserver, the per-channel observer / quantizer, "
            "QuantizationManager, FakeQuantize); the multi-tensor, fused-kernel and LSQFakeQuantize "
            "kernels need the GPU.")
    if x.dtype != torch.float32:
        raise TypeError(f"{what}: only float32 is supported by the HIP fake-quant path, got {x.dtype}")
    return x.contiguous()


def mask_buffer(rows: int, rowlen: int, device) -> torch.Tensor:
    """1-bit straight-through mask storage (uint64 words, layout in include/vsiq.h)."""
    words = int(lib().vsiq_mask_words(int(rows), int(rowlen)))
    return torch.empty(max(words, 1), dtype=torch.int64, device=device)


def set_tuning(key: int, value: int):
    check(lib().vsiq_set_tuning(int(key), int(value)), "vsiq_set_tuning")


def gate_tuning_pending() -> int:
    """Store-gate launch sites still tuning (vsiq_gate_tuning_pending)."""
    return int(lib().vsiq_gate_tuning_pending())


def gate_retune() -> int:
    """Re-tune every store-gate launch site (vsiq_gate_retune); returns the site count."""
    return int(lib().vsiq_gate_retune())


def gate_report() -> str:
    """One line per tuned store-gate launch site (vsiq_gate_report)."""
    n = int(lib().vsiq_gate_report(None, 0))
    buf = ctypes.create_string_buffer(n + 1)
    lib().vsiq_gate_report(buf, n + 1)
    return buf.value.decode()


def gate_export() -> str:
    """The tuned store-gate table, one "<kernel symbol> <grid> <bytes> <ticks>" line per
    site (vsiq_gate_export)."""
    n = int(lib().vsiq_gate_export(None, 0))
    buf = ctypes.create_string_buffer(n + 1)
    lib().vsiq_gate_export(buf, n + 1)
    return buf.value.decode()


def gate_import(text: str) -> int:
    """Load gate_export's lines: a listed site takes that gate and is never timed."""
    n = int(lib().vsiq_gate_import(text.encode()))
    if n < 0:
        raise ValueError("vsiq_gate_import: malformed gate table")
    return n


def gate_freeze(on: bool = True) -> bool:
    """Stop (or resume) all store-gate timing; returns the previous setting."""
    return bool(lib().vsiq_gate_freeze(int(bool(on))))


def gate_save(path: str) -> int:
    """Write the tuned gate table to `path`; returns the number of sites."""
    text = gate_export()
    with open(path, "w") as f:
        f.write(text)
    return text.count("\n")


def gate_load(path: str, freeze: bool = True) -> int:
    """Load a table written by gate_save and (default) freeze the tuner: reproducible
    timing, no candidate launches.  Returns the number of loaded sites."""
    with open(path) as f:
        n = gate_import(f.read())
    if freeze:
        gate_freeze(True)
    return n


def ptr(t):
    return None if t is None else c_p(t.data_ptr())


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(device) -> c_p:
    """torch's current HIP stream on `device` (the raw handle; ~0.3 us instead of the ~2 us
    of building a torch.cuda.Stream object per launch)."""
    if _RAW_STREAM is not None:
        idx = device.index if isinstance(device, torch.device) else device
        if idx is None:
            idx = torch.cuda.current_device()
        return c_p(_RAW_STREAM(idx))
    return c_p(torch.cuda.current_stream(device).cuda_stream)


class _Workspace:
    """Per (device, stream) reduction workspace + self-resetting arrival counter."""

    def __init__(self, device, n):
        self.device = device
        self.counter = torch.zeros(COUNTER_WORDS, dtype=torch.int32, device=device)
        self.ws = None
        self.ws_len = 0
        self.reserve(n)

    def reserve(self, n):
        return self.reserve_doubles(int(lib().vsiq_workspace_doubles(int(n))))

    def reserve_doubles(self, need):
        if need > self.ws_len:
            self.ws = torch.empty(need, dtype=torch.float64, device=self.device)
            self.ws_len = need
        return self

    def channel_counters(self, channels: int) -> torch.Tensor:
        """Per-channel arrival counters (zeroed once; every launch leaves them zero)."""
        c = getattr(self, "_chan", None)
        if c is None or c.numel() < channels:
            c = self._chan = torch.zeros(max(channels, 256), dtype=torch.int32, device=self.device)
        return c


_WS = {}
_HIPRT = []


def _capture_id(stream: c_p):
    """hipStreamGetCaptureInfo id of the capture `stream` is in, or None."""
    if not _HIPRT:
        rt = ctypes.CDLL("libamdhip64.so")
        rt.hipStreamGetCaptureInfo.argtypes = [c_p, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_ulonglong)]
        rt.hipStreamGetCaptureInfo.restype = c_int
        _HIPRT.append(rt)
    status, cid = c_int(0), ctypes.c_ulonglong(0)
    if _HIPRT[0].hipStreamGetCaptureInfo(stream, ctypes.byref(status), ctypes.byref(cid)) != 0:
        return None
    return cid.value if status.value == 1 else None   # hipStreamCaptureStatusActive


def workspace(device, n: int = 0) -> _Workspace:
    """Workspace for a reducing launch over n elements on the current stream of `device`.
    (Growing it while a previous launch still reads the old buffer is safe: the caching
    allocator only recycles the old block after work queued on this stream.)  Under
    HIP-graph capture the key is the capture: every graph gets its own workspace and
    counter (allocated from its pool), so graphs replayed concurrently on different
    streams never share a counter."""
    dev = torch.device(device)
    st = stream_of(dev)
    key = (dev.index, st.value)
    if torch.cuda.is_current_stream_capturing():
        key = (dev.index, "capture", _capture_id(st))
    w = _WS.get(key)
    if w is None:
        w = _WS[key] = _Workspace(dev, n)
    return w.reserve(n)
