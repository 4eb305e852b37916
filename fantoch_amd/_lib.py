"""ctypes binding of libbote_hip.so (include/bote_hip.h).

The library is built in-tree (fantoch_amd/lib/libbote_hip.so) by
`__graft_entry__.build()` / `make -C fantoch_amd/csrc`.  There is no CPU
fallback: if the library is missing, every product entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BOTE_LIB_PATH: an alternative in-tree build for A/B timing experiments
LIB_PATH = os.environ.get("BOTE_LIB_PATH") or os.path.join(HERE, "lib", "libbote_hip.so")
CSRC = os.path.join(HERE, "csrc")
INCLUDE_H = os.path.join(os.path.dirname(HERE), "include", "bote_hip.h")

BOTE_OK = 0
ERRORS = {-1: "BOTE_E_ARG", -2: "BOTE_E_QUORUM_GT_N", -3: "BOTE_E_DEVICE", -4: "BOTE_E_RANGE",
          -5: "BOTE_E_NOMEM", -6: "BOTE_E_NODEV"}

FPAXOS, EPAXOS, ATLAS, TEMPO, TEMPO_TINY = 0, 1, 2, 3, 4
STAT_MEAN, STAT_COV, STAT_MDTM = 0, 1, 2
SLOT_AF1, SLOT_FF1, SLOT_AF2, SLOT_FF2, SLOT_E = 0, 1, 2, 3, 4
SLOT_NAMES = ["af1", "ff1", "af2", "ff2", "e", "af1C", "ff1C", "af2C", "ff2C", "eC"]
# the extended key set (BOTE_KEYS_TEMPO_ALL_LEADERS, include/bote_hip.h)
KEYS_BASE, KEYS_TEMPO_ALL_LEADERS = 0, 1
SLOT_TT1, SLOT_TT2, SLOT_TW1, SLOT_TW2, SLOT_FL1, SLOT_FL2 = 10, 11, 12, 13, 18, 19
SLOT_X_COLOCATED = 4
NSLOTS_X = 20
SLOT_NAMES_X = SLOT_NAMES + ["ttf1", "ttf2", "twf1", "twf2", "ttf1C", "ttf2C", "twf1C", "twf2C", "fl1", "fl2"]
OBJ_SCORE, OBJ_MEAN, OBJ_COV = 0, 1, 2
FT_F1, FT_F1F2 = 1, 2
KP = 128

# Every symbol declared in include/bote_hip.h (checked by tests/test_abi.py).
EXPORTS = [
    "bote_last_error", "bote_device_count", "bote_planet_create", "bote_planet_destroy",
    "bote_planet_regions", "bote_quorum_size", "bote_max_f", "bote_quorum_latencies",
    "bote_leaderless", "bote_leader", "bote_all_leaders", "bote_best_leader", "bote_eval",
    "bote_sweep_create", "bote_sweep_launch", "bote_sweep_result", "bote_sweep_result_bytes",
    "bote_sweep_result_device", "bote_merge_device", "bote_sweep_last_kernel_ms",
    "bote_sweep_destroy", "bote_colex_unrank", "bote_binomial", "bote_sweep_timing_reset",
    "bote_sweep_timing", "bote_sweep_grid", "bote_sweep_is_fast", "bote_sweep_split", "bote_sweep_create_ex", "bote_search_topk", "bote_sweep_deferred", "bote_eval_leaderless", "bote_evolving_chains",
    "bote_search_create", "bote_search_launch", "bote_search_result", "bote_search_bounds", "bote_search_destroy",
    "bote_eval_keys", "bote_sweep_create_keys",
]
KERNELS = {None: 0, "auto": 0, "generic": 1, "fast": 2, "group": 3}


class BoteError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class Objective(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("slot", C.c_uint32)]


class RankingParamsC(C.Structure):
    _fields_ = [("min_mean_fpaxos_improv", C.c_double), ("min_mean_epaxos_improv", C.c_double),
                ("min_fairness_fpaxos_improv", C.c_double), ("min_mean_decrease", C.c_double),
                ("ft_metric", C.c_int32)]


class TopKRecord(C.Structure):
    _fields_ = [("key", C.c_uint64), ("rank", C.c_uint64)]


_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_vp = C.c_void_p

_LIB = None


def build(jobs: int = 2) -> str:
    """Compile libbote_hip.so for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", CSRC, f"-j{jobs}"], check=True)
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {CSRC}` "
                          "(there is no CPU fallback for the HIP path)")
    # One HIP runtime per process: PyTorch ROCm bundles libamdhip64 (soname
    # libamdhip64.so.7) and needs it under its unversioned name, so once
    # /opt/rocm's copy is loaded first torch finds no device.  Loading torch
    # first makes our DT_NEEDED libamdhip64.so.7 resolve to the same runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    L.bote_last_error.restype = C.c_char_p
    L.bote_device_count.argtypes = [C.POINTER(C.c_int)]
    L.bote_planet_create.argtypes = [_u16p, C.c_uint32, C.c_int, C.POINTER(_vp)]
    L.bote_planet_destroy.argtypes = [_vp]
    L.bote_planet_regions.argtypes = [_vp, C.POINTER(C.c_uint32)]
    L.bote_quorum_size.argtypes = [C.c_int, C.c_uint32, C.c_uint32]
    L.bote_max_f.restype = C.c_uint32
    L.bote_max_f.argtypes = [C.c_uint32]
    L.bote_quorum_latencies.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32, _u64p]
    L.bote_leaderless.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32, _u64p]
    L.bote_leader.argtypes = [_vp, C.c_uint32, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32, _u64p]
    L.bote_all_leaders.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32, _u64p]
    L.bote_best_leader.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32, C.c_int,
                                   C.POINTER(C.c_uint32), _vp]
    L.bote_eval.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32, _vp, C.c_uint64,
                            C.c_uint64, C.POINTER(RankingParamsC), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.bote_eval_leaderless.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32, _vp, C.c_uint64,
                                       C.c_uint64, _u32p, C.c_uint32, _vp, _vp, _vp]
    L.bote_evolving_chains.argtypes = [C.c_int, C.c_uint32, _u32p, _vp, _vp, _vp, C.c_double, C.c_int, C.c_uint64,
                                       _vp, _vp, C.POINTER(C.c_uint64)]
    L.bote_sweep_create.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32,
                                    C.POINTER(Objective), C.c_uint32, C.c_uint32,
                                    C.POINTER(RankingParamsC), C.c_int, C.POINTER(_vp)]
    L.bote_sweep_create_ex.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32,
                                       C.POINTER(Objective), C.c_uint32, C.c_uint32,
                                       C.POINTER(RankingParamsC), C.c_int, C.c_int, C.POINTER(_vp)]
    L.bote_eval_keys.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32, _vp, C.c_uint64, C.c_uint64,
                                 C.c_uint32, _vp, _vp, _vp, _vp, _vp]
    L.bote_sweep_create_keys.argtypes = [_vp, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32,
                                         C.POINTER(Objective), C.c_uint32, C.c_uint32,
                                         C.POINTER(RankingParamsC), C.c_int, C.c_int, C.c_uint32, C.POINTER(_vp)]
    L.bote_search_topk.argtypes = [C.POINTER(_vp), C.c_uint32, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32,
                                   C.c_uint64, C.c_uint64, C.POINTER(Objective), C.c_uint32, C.c_uint32,
                                   C.POINTER(RankingParamsC), C.c_int, C.POINTER(TopKRecord), _vp,
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.bote_search_create.argtypes = [C.POINTER(_vp), C.c_uint32, _u32p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32,
                                     C.c_uint64, C.c_uint64, C.POINTER(Objective), C.c_uint32, C.c_uint32,
                                     C.POINTER(RankingParamsC), C.c_int, C.c_uint32, C.POINTER(_vp)]
    L.bote_search_launch.argtypes = [_vp]
    L.bote_search_result.argtypes = [_vp, C.POINTER(TopKRecord), _vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.bote_search_bounds.argtypes = [_vp, C.POINTER(C.c_uint64)]
    L.bote_search_destroy.argtypes = [_vp]
    L.bote_sweep_launch.argtypes = [_vp, C.c_uint64, C.c_uint64, _vp]
    L.bote_sweep_result.argtypes = [_vp, _vp, C.POINTER(TopKRecord), _vp, C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint64)]
    L.bote_sweep_result_bytes.restype = C.c_uint64
    L.bote_sweep_result_bytes.argtypes = [_vp]
    L.bote_sweep_result_device.argtypes = [_vp, _vp, _vp]
    L.bote_merge_device.argtypes = [_vp, _vp, C.c_uint32, _vp, _vp]
    L.bote_sweep_last_kernel_ms.argtypes = [_vp, C.POINTER(C.c_float)]
    L.bote_sweep_destroy.argtypes = [_vp]
    L.bote_sweep_timing_reset.argtypes = [_vp]
    L.bote_sweep_timing.argtypes = [_vp, C.POINTER(C.c_float), C.POINTER(C.c_uint32)]
    L.bote_sweep_grid.argtypes = [_vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.bote_sweep_is_fast.argtypes = [_vp, C.POINTER(C.c_int)]
    L.bote_sweep_split.argtypes = [_vp, C.c_uint64, C.c_uint64, C.c_uint32, C.POINTER(C.c_uint64)]
    L.bote_sweep_deferred.argtypes = [_vp, _vp, C.POINTER(C.c_uint64)]
    L.bote_colex_unrank.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, _u32p]
    L.bote_binomial.restype = C.c_uint64
    L.bote_binomial.argtypes = [C.c_uint32, C.c_uint32]
    _LIB = L
    return L


def check(rc: int):
    if rc != BOTE_OK:
        raise BoteError(rc, lib().bote_last_error().decode())


def u32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32).reshape(-1))


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def ranking_params_c(rp) -> RankingParamsC:
    return RankingParamsC(float(rp.min_mean_fpaxos_improv), float(rp.min_mean_epaxos_improv),
                          float(rp.min_fairness_fpaxos_improv), float(rp.min_mean_decrease),
                          int(rp.ft_metric.value))


def device_count() -> int:
    n = C.c_int(0)
    check(lib().bote_device_count(C.byref(n)))
    return n.value


def binomial(ns: int, n: int) -> int:
    return int(lib().bote_binomial(ns, n))


def colex_unrank(rank: int, n: int, ns: int) -> np.ndarray:
    out = np.zeros(n, np.uint32)
    check(lib().bote_colex_unrank(rank, n, ns, out))
    return out
