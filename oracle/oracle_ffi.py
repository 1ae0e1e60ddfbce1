"""ORACLE — TEST INFRASTRUCTURE ONLY (ctypes binding of oracle/build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
Also holds an independent numpy parser of the reference fixture key
(test_data/client_key, bincode 1.3.3 layout) so that the
product's C++ parser is cross-checked against a second implementation.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")  # x86-64-v3 (AVX2 + FMA)
LIB_PATH_V2 = os.path.join(HERE, "build", "liboracle_v2.so")  # the same source for CPUs without FMA


def _cpu_has_fma() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    fl = set(line.split(":", 1)[1].split())
                    return {"fma", "avx2"} <= fl
    except OSError:
        pass
    return False
Q_RING = 998244353 * 1004535809  # GLWE/GGSW ring modulus (RNS: two NTT primes)
RNS_PRIMES = (998244353, 1004535809)


class Params(C.Structure):
    _fields_ = [("k", C.c_int32), ("N", C.c_int32), ("n", C.c_int32), ("ks_base_log", C.c_int32),
                ("ks_level", C.c_int32), ("pbs_base_log", C.c_int32), ("pbs_level", C.c_int32),
                ("ring", C.c_int32), ("lwe_sigma", C.c_double), ("glwe_sigma", C.c_double)]


class Gate(C.Structure):
    _fields_ = [("n_in", C.c_int32), ("offset", C.c_int32), ("in_idx", C.c_int32 * 16),
                ("in_w", C.c_int32 * 16), ("n_out", C.c_int32), ("direct", C.c_int32),
                ("lut", (C.c_uint8 * 16) * 8)]


def lut_terms(N: int, lut) -> list:
    """w_f of the multi-value factorization: [(position, coefficient)]."""
    box, half = N // 16, N // 32
    t = [(m * box - half, int(lut[m]) - int(lut[m - 1])) for m in range(1, 16) if lut[m] != lut[m - 1]]
    dd = -(int(lut[0]) + int(lut[15]))
    if dd:
        t.append((N - half, dd))
    return t


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = LIB_PATH if _cpu_has_fma() else LIB_PATH_V2
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        u64p = C.POINTER(C.c_uint64)
        L.or_q_mul.restype = C.c_uint64
        L.or_q_mul.argtypes = [C.c_uint64, C.c_uint64]
        L.or_q_modulus.restype = C.c_uint64
        L.or_pbs_gadget.restype = C.c_uint64
        L.or_rng_u64.restype = C.c_uint64
        L.or_rng_u64.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.or_gaussian.restype = C.c_int64
        L.or_gaussian.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_double]
        L.or_ring_mul.argtypes = [C.c_int, u64p, u64p, u64p]
        L.or_ring_mul_schoolbook.argtypes = [C.c_int, u64p, u64p, u64p]
        L.or_decompose_pbs.restype = C.c_uint64
        L.or_decompose_pbs.argtypes = [C.c_uint64]
        L.or_conv.restype = C.c_uint64
        L.or_conv.argtypes = [C.c_uint64]
        L.or_ks_decompose.argtypes = [C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_int32)]
        L.or_mod_switch.restype = C.c_uint32
        L.or_mod_switch.argtypes = [C.c_uint64, C.c_int]
        L.or_keygen_ksk.argtypes = [C.POINTER(Params), u64p, u64p, C.c_uint64, u64p]
        L.or_keygen_bsk.argtypes = [C.POINTER(Params), u64p, u64p, C.c_uint64, u64p]
        L.or_bsk_len.restype = C.c_size_t
        L.or_bsk_len.argtypes = [C.POINTER(Params)]
        L.or_bsk_unroll.argtypes = [C.POINTER(Params)]
        L.or_encrypt.argtypes = [C.POINTER(Params), u64p, C.POINTER(C.c_uint8), C.c_size_t, C.c_uint64, C.c_uint64, u64p]
        L.or_phase.argtypes = [C.c_int, u64p, u64p, C.c_size_t, u64p]
        L.or_decode16.restype = C.c_uint32
        L.or_decode16.argtypes = [C.c_uint64]
        L.or_keyswitch.argtypes = [C.POINTER(Params), u64p, u64p, C.c_size_t, u64p]
        L.or_bsk_prepare.restype = C.c_void_p
        L.or_bsk_prepare.argtypes = [C.POINTER(Params), u64p]
        L.or_bsk_free.argtypes = [C.c_void_p]
        L.or_blind_rotate.argtypes = [C.c_void_p, u64p, C.POINTER(C.c_uint8), u64p]
        L.or_blind_rotate_multi.argtypes = [C.c_void_p, u64p, C.POINTER(C.c_uint8), C.c_int, C.c_int, u64p]
        L.or_lut_terms.restype = C.c_int
        L.or_lut_terms.argtypes = [C.c_int, C.POINTER(C.c_uint8), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.or_lincomb.argtypes = [C.c_int, C.POINTER(Gate), u64p, u64p]
        L.or_gates.argtypes = [C.c_void_p, u64p, C.POINTER(Gate), C.c_size_t, u64p, C.POINTER(C.c_int32), u64p]
        L.or_fft_ring_mul.argtypes = [C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.or_fft_tables.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint16)]
        L.or_bsk_fourier.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        L.or_torus_of.restype = C.c_uint64
        L.or_torus_of.argtypes = [C.c_double]
        L.or_blind_rotate_exact.argtypes = [C.POINTER(Params), u64p, u64p, C.POINTER(C.c_uint8), C.c_int, C.c_int,
                                            C.c_size_t, u64p]
        L.or_num_threads.restype = C.c_int
        L.or_set_threads.argtypes = [C.c_int]
        _lib = L
    return _lib


def ptr(a: np.ndarray, t=C.c_uint64):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(t))


# ----------------------------------------------------------- fixture key parse
def parse_client_key(blob: bytes) -> dict:
    """Second, independent parser of the bincode RadixClientKey."""
    u = lambda off: struct.unpack_from("<Q", blob, off)[0]
    n_big = u(0)
    s_big = np.frombuffer(blob, dtype="<u8", count=n_big, offset=8).copy()
    off = 8 + 8 * n_big
    n_glwe = u(off)
    glwe = np.frombuffer(blob, dtype="<u8", count=n_glwe, offset=off + 8).copy()
    off += 8 + 8 * n_glwe
    poly_size = u(off); off += 8
    n_small = u(off)
    s_small = np.frombuffer(blob, dtype="<u8", count=n_small, offset=off + 8).copy()
    off += 8 + 8 * n_small
    lwe_dim, glwe_dim, N = u(off), u(off + 8), u(off + 16)
    lwe_sigma, glwe_sigma = struct.unpack_from("<dd", blob, off + 24)
    pbs_base_log, pbs_level, ks_base_log, ks_level = (u(off + 40), u(off + 48), u(off + 56), u(off + 64))
    msg_mod, carry_mod = u(off + 112), u(off + 120)
    num_blocks = u(off + 128)
    assert off + 136 == len(blob)
    return dict(s_big=s_big, glwe=glwe, poly_size=poly_size, s_small=s_small, n=lwe_dim, k=glwe_dim, N=N,
                lwe_sigma=lwe_sigma, glwe_sigma=glwe_sigma, pbs_base_log=pbs_base_log, pbs_level=pbs_level,
                ks_base_log=ks_base_log, ks_level=ks_level, message_modulus=msg_mod, carry_modulus=carry_mod,
                num_blocks=num_blocks)


RING_RNS, RING_FFT = 0, 1  # fheregex.h FR_RING_*


def params_from_key(key: dict, k: int | None = None, N: int | None = None, ring: int | None = None) -> Params:
    """Reference params (k=1, N=2048) or the k=2, N=1024 reinterpretation of the
    same 2048-bit flattened GLWE key; ring: RING_FFT (2^64
    torus, f64 FFT as tfhe-rs; the product's default at both points) or
    RING_RNS (Z_Q, NTT)."""
    k = int(key["k"]) if k is None else k
    N = int(key["N"]) if N is None else N
    if ring is None:
        ring = RING_FFT if (k, N) in ((1, 2048), (2, 1024)) else RING_RNS
    assert k * N == len(key["s_big"])
    return Params(k, N, int(key["n"]), int(key["ks_base_log"]), int(key["ks_level"]),
                  int(key["pbs_base_log"]), int(key["pbs_level"]), ring, float(key["lwe_sigma"]),
                  float(key["glwe_sigma"]))


class Oracle:
    """Keys + helpers around liboracle for a parameter set."""

    def __init__(self, key: dict, seed: int, k: int | None = None, N: int | None = None, with_bsk=True,
                 ring: int | None = None):
        self.key = key
        self.P = params_from_key(key, k, N, ring)
        self.seed = seed
        self.big = self.P.k * self.P.N
        self.n = self.P.n
        L = lib()
        self.s_big = np.ascontiguousarray(key["s_big"], dtype=np.uint64)
        self.s_small = np.ascontiguousarray(key["s_small"], dtype=np.uint64)
        self.ksk = np.zeros(self.big * self.P.ks_level * (self.n + 1), dtype=np.uint64)
        L.or_keygen_ksk(C.byref(self.P), ptr(self.s_big), ptr(self.s_small), seed, ptr(self.ksk))
        self.bsk = None
        self._pk = None
        if with_bsk:
            self.bsk = np.zeros(L.or_bsk_len(C.byref(self.P)), dtype=np.uint64)
            L.or_keygen_bsk(C.byref(self.P), ptr(self.s_big), ptr(self.s_small), seed, ptr(self.bsk))
            self._pk = L.or_bsk_prepare(C.byref(self.P), ptr(self.bsk))

    def bsk_fourier(self) -> np.ndarray:
        """Fourier-domain BSK (torus ring): [w][r][c][slot] complex128, scaled by 1/M."""
        assert self.P.ring == RING_FFT and self._pk
        M = self.P.N // 2
        out = np.zeros(len(self.bsk) // self.P.N * M * 2, dtype=np.float64)
        lib().or_bsk_fourier(self._pk, ptr(out, C.c_double))
        return out.view(np.complex128)

    def __del__(self):
        if getattr(self, "_pk", None):
            lib().or_bsk_free(self._pk)
            self._pk = None

    # -- client side
    def encrypt_blocks(self, msgs, seed: int, first_block: int = 0) -> np.ndarray:
        m = np.ascontiguousarray(np.asarray(msgs, dtype=np.uint8))
        out = np.zeros((len(m), self.big + 1), dtype=np.uint64)
        lib().or_encrypt(C.byref(self.P), ptr(self.s_big), ptr(m, C.c_uint8), len(m), seed, first_block, ptr(out))
        return out

    def encrypt_str(self, s: bytes, seed: int) -> np.ndarray:
        """Radix encoding of src/regex/ciphertext.rs:18-29 (base-4 digits, LSB first)."""
        msgs = [(b >> (2 * i)) & 3 for b in s for i in range(4)]
        return self.encrypt_blocks(msgs, seed).reshape(len(s), 4, self.big + 1)

    def trivial_blocks(self, msgs) -> np.ndarray:
        m = np.asarray(msgs, dtype=np.uint64)
        out = np.zeros((len(m), self.big + 1), dtype=np.uint64)
        out[:, -1] = m << np.uint64(59)
        return out

    def phase(self, lwe: np.ndarray, key=None) -> np.ndarray:
        s = self.s_big if key is None else key
        a = np.ascontiguousarray(lwe.reshape(-1, len(s) + 1), dtype=np.uint64)
        out = np.zeros(a.shape[0], dtype=np.uint64)
        lib().or_phase(len(s), ptr(np.ascontiguousarray(s, dtype=np.uint64)), ptr(a), a.shape[0], ptr(out))
        return out

    def decode16(self, lwe: np.ndarray) -> np.ndarray:
        return np.array([lib().or_decode16(int(x)) for x in self.phase(lwe)], dtype=np.uint32)

    def decrypt_radix(self, blocks: np.ndarray) -> int:
        """RadixClientKey::decrypt: sum (block msg mod 4) * 4^i."""
        d = self.decode16(blocks.reshape(-1, self.big + 1))
        return int(sum(int(v % 4) << (2 * i) for i, v in enumerate(d))) & 0xFF

    # -- server side
    def keyswitch(self, lwe: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(lwe.reshape(-1, self.big + 1), dtype=np.uint64)
        out = np.zeros((a.shape[0], self.n + 1), dtype=np.uint64)
        lib().or_keyswitch(C.byref(self.P), ptr(self.ksk), ptr(a), a.shape[0], ptr(out))
        return out

    def blind_rotate(self, ks_lwe: np.ndarray, lut) -> np.ndarray:
        l = (C.c_uint8 * 16)(*lut)
        out = np.zeros(self.big + 1, dtype=np.uint64)
        a = np.ascontiguousarray(ks_lwe, dtype=np.uint64)
        lib().or_blind_rotate(self._pk, ptr(a), l, ptr(out))
        return out

    def blind_rotate_multi(self, ks_lwe: np.ndarray, luts, direct: bool = False) -> np.ndarray:
        luts = [list(l) for l in luts]
        assert 1 <= len(luts) <= 8 and (not direct or len(luts) == 1)
        flat = (C.c_uint8 * (16 * len(luts)))(*[v for l in luts for v in l])
        out = np.zeros((len(luts), self.big + 1), dtype=np.uint64)
        a = np.ascontiguousarray(ks_lwe, dtype=np.uint64)
        lib().or_blind_rotate_multi(self._pk, ptr(a), flat, len(luts), int(direct), ptr(out))
        return out

    def blind_rotate_exact(self, ks_lwes: np.ndarray, luts, direct: int = 1) -> np.ndarray:
        """The torus ring's unrolled ladder in exact u64 arithmetic (schoolbook negacyclic
        products mod 2^64, no f64): ks_lwes (count, n+1); luts (count, n_out, 16) or
        (count, 16) for direct jobs; returns (count, n_out, kN+1)."""
        assert self.P.ring == RING_FFT and self.bsk is not None
        a = np.ascontiguousarray(ks_lwes.reshape(-1, self.n + 1), dtype=np.uint64)
        count = a.shape[0]
        l = np.ascontiguousarray(np.asarray(luts, dtype=np.uint8).reshape(count, -1, 16))
        n_out = 1 if direct else l.shape[1]
        out = np.zeros((count, n_out, self.big + 1), dtype=np.uint64)
        lib().or_blind_rotate_exact(C.byref(self.P), ptr(self.bsk), ptr(a), ptr(l, C.c_uint8), l.shape[1], int(direct),
                                    count, ptr(out))
        return out

    def gates(self, gates, slots: np.ndarray) -> np.ndarray:
        """gates: list of (inputs [(slot, weight)], offset, luts, direct) jobs, offset
        in units of Delta/2; a bare 16-entry lut means one direct output; direct=2
        is a sign gate (luts ignored).  Returns all outputs, job-major."""
        arr = (Gate * len(gates))()
        first = (C.c_int32 * len(gates))()
        total = 0
        for q, job in enumerate(gates):
            ins, off, luts = job[0], job[1], job[2]
            direct = job[3] if len(job) > 3 else None
            if len(luts) == 16 and not isinstance(luts[0], (list, tuple)):
                luts, direct = [luts], 1 if direct is None else direct
            g = arr[q]
            g.n_in = len(ins)
            g.offset = off
            for t, (i, w) in enumerate(ins):
                g.in_idx[t] = i
                g.in_w[t] = w
            g.n_out = len(luts)
            g.direct = int(direct or 0)
            for f, lut in enumerate(luts):
                for t in range(16):
                    g.lut[f][t] = lut[t]
            first[q] = total
            total += len(luts)
        s = np.ascontiguousarray(slots.reshape(-1, self.big + 1), dtype=np.uint64)
        out = np.zeros((total, self.big + 1), dtype=np.uint64)
        lib().or_gates(self._pk, ptr(self.ksk), arr, len(gates), ptr(s), first, ptr(out))
        return out

    def run_schedule(self, S, content_lwes: np.ndarray, levels=None) -> np.ndarray:
        """Evaluate a match schedule (fheregex.schedule_match: fr_job semantics)
        level by level, each level's jobs in one parallel or_gates call; returns
        the result LWE (block 0 of the boolean).  levels: optional range of levels
        (the caller then reads self.sched_val)."""
        content = content_lwes.reshape(-1, self.big + 1)
        if levels is None:
            self.sched_val = {}
            levels = range(len(S.level_off) - 1)
        val = self.sched_val
        for l in levels:
            rows, index, jobs = [], {}, []
            js = S.jobs[S.level_off[l]:S.level_off[l + 1]]
            for j in js:
                ins = []
                for q in range(j.n_in):
                    r = j.in_ref[q]
                    if r not in index:
                        index[r] = len(rows)
                        rows.append(val[r] if r >= 0 else content[-1 - r])
                    ins.append((index[r], j.in_w[q]))
                jobs.append((ins, j.offset, [list(j.lut[f]) for f in range(j.n_out)], j.kind))
            outs = self.gates(jobs, np.stack(rows))
            k = 0
            for j in js:
                for f in range(j.n_out):
                    val[j.out_gate[f]] = outs[k]
                    k += 1
        return self._output(S.out_gate, S.out_w, S.out_const)

    def _output(self, gate, w, cst) -> np.ndarray:
        """a program output cst + w * gate from the last run's gate values (a linear op)"""
        out = np.zeros(self.big + 1, dtype=np.uint64)
        if gate >= 0:
            out = (np.uint64(w & 0xFFFFFFFFFFFFFFFF) * self.sched_val[gate]).astype(np.uint64)
        out[-1] += np.uint64((cst << 59) & 0xFFFFFFFFFFFFFFFF)
        return out

    def run_schedule_parts(self, S, content_lwes: np.ndarray) -> list:
        """run_schedule of a parts schedule (fheregex.schedule_match max_parts > 1): the
        LWE of every part"""
        self.run_schedule(S, content_lwes)
        return [self._output(*p) for p in S.parts]

    @staticmethod
    def set_threads(t: int):
        lib().or_set_threads(t)

    @staticmethod
    def num_threads() -> int:
        return lib().or_num_threads()


def load_fixture_key(path: str | None = None) -> dict:
    if path is None:
        path = os.path.join(os.path.dirname(HERE), "tests", "golden", "client_key")
    with open(path, "rb") as f:
        return parse_client_key(f.read())
