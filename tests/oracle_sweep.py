"""TEST INFRASTRUCTURE: an oracle-backed stand-in for fantoch_amd.bote.Sweep
with the same block interface (launch / result_bytes / result_device /
merge_device / parse_block), so the multi-rank orchestration in
fantoch_amd/dist.py can run under gloo on CPU.  The block layout is the device
one (include/bote_hip.h, bote_sweep_result_device): n_obj x 128 records of
(key u64, rank u64), ascending, padded with all-ones, then valid u64 and
digest u64."""
import ctypes as C
from math import comb

import numpy as np

import oracle as O
from fantoch_amd import _lib
from fantoch_amd.bote import Sweep

KP = _lib.KP
PAD = 0xFFFFFFFFFFFFFFFF


def merge_blocks(blocks, n_obj):
    """Host restatement of merge_kernel + sum_counters_kernel."""
    out = np.full(n_obj * KP * 2 + 2, PAD, dtype=np.uint64)
    for o in range(n_obj):
        recs = []
        for b in blocks:
            r = b[o * KP * 2:(o + 1) * KP * 2].reshape(KP, 2)
            recs.extend((int(k), int(x)) for k, x in r if not (k == PAD and x == PAD))
        recs.sort()
        for i, (k, x) in enumerate(recs[:KP]):
            out[(o * KP + i) * 2] = k
            out[(o * KP + i) * 2 + 1] = x
    out[n_obj * KP * 2] = sum(int(b[n_obj * KP * 2]) for b in blocks) % (1 << 64)
    out[n_obj * KP * 2 + 1] = sum(int(b[n_obj * KP * 2 + 1]) for b in blocks) % (1 << 64)
    return out


class OracleSweep:
    def __init__(self, oplanet, servers, clients, n, objectives, K, rparams=(110.0, 35.0, 0.0, 15.0), keys=0,
                 threads=2):
        self.o, self.n, self.K, self.keys, self.threads = oplanet, n, K, keys, threads
        self.servers = np.asarray(servers, dtype=np.uint32)
        self.clients = np.asarray(clients, dtype=np.uint32)
        self.objectives = list(objectives)
        self.rparams = rparams
        self.total = comb(len(self.servers), n)
        self._blk = None

    def launch(self, rb, re, stream=None):
        tops, valid, digest = self.o.sweep(self.servers, self.clients, self.n, rb, re, self.objectives, self.K,
                                           self.rparams, 2, self.threads, keys=self.keys)
        no = len(self.objectives)
        blk = np.full(no * KP * 2 + 2, PAD, dtype=np.uint64)
        for o, lst in enumerate(tops):
            for i, (k, x) in enumerate(lst):
                blk[(o * KP + i) * 2] = k
                blk[(o * KP + i) * 2 + 1] = x
        blk[no * KP * 2] = valid
        blk[no * KP * 2 + 1] = digest
        self._blk = blk

    def result_bytes(self):
        return (len(self.objectives) * KP * 2 + 2) * 8

    def result_device(self, ptr, stream=None):
        C.memmove(ptr, self._blk.ctypes.data, self.result_bytes())

    def merge_device(self, src, n, dst, stream=None):
        nb = self.result_bytes()
        raw = np.frombuffer(C.string_at(src, n * nb), dtype=np.uint64)
        blocks = [raw[i * (nb // 8):(i + 1) * (nb // 8)] for i in range(n)]
        out = merge_blocks(blocks, len(self.objectives))
        C.memmove(dst, out.ctypes.data, nb)

    def parse_block(self, blk):
        return Sweep.parse_block(self, blk)
