"""Python mirror of the reference's regex API over the MI355X C-ABI (libfheregex.so).

Reference API (RKlompUU/fhe-regex) -> here:
  src/regex/ciphertext.rs:42-45  gen_keys()                    -> gen_keys(...)
  src/regex/ciphertext.rs:32-40  encrypt_str(ck, s)            -> ClientKey.encrypt_str(s)
  src/regex/ciphertext.rs:8-30   create_trivial_radix(sk, m)   -> ServerKey.create_trivial_radix(m)
  src/regex/engine.rs:8-42       has_match(sk, content, pat)   -> has_match(sk, content, pat)
  RadixClientKey::decrypt                                      -> ClientKey.decrypt(ct)
  src/regex/parser.rs:146-185    parse(pattern)                -> parse(pattern) (canonical AST string)

Errors mirror the reference: a pattern the reference rejects raises ``ParseError``
(reference: ``Err``), a pattern/content on which the reference panics raises
``ReferencePanic``, non-ASCII content raises ``ValueError`` (ciphertext.rs:33-35).

All homomorphic work runs in the HIP kernels behind the C-ABI; there is no CPU
fallback: a GPU op on a context without a device raises ``NoDevice``.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Tuple, List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FHEREGEX_LIB") or os.path.join(HERE, "libfheregex.so")
REPO = os.path.dirname(HERE)
HEADER = os.path.join(REPO, "include", "fheregex.h")

FR_OK = 0
ERR_INVALID, ERR_PARSE, ERR_REF_PANIC, ERR_NO_DEVICE, ERR_HIP, ERR_NO_KEY, ERR_OOM, ERR_NON_ASCII = range(-1, -9, -1)
LOWER_FAITHFUL, LOWER_THRESHOLD, LOWER_FAITHFUL_TREE = 0, 1, 2
ENGINE_AUTO, ENGINE_ENUMERATE, ENGINE_MERGED = 0, 1, 2
GRAMMAR_REFERENCE, GRAMMAR_EXT = 0, 1
KEYGEN_AUTO, KEYGEN_HOST, KEYGEN_DEVICE = 0, 1, 2
NULL_CT = 0xFFFFFFFF


class FheRegexError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class ParseError(FheRegexError):
    pass


class ReferencePanic(FheRegexError):
    pass


class NoDevice(FheRegexError):
    pass


class Params(C.Structure):
    _fields_ = [("k", C.c_int32), ("N", C.c_int32), ("n", C.c_int32), ("ks_base_log", C.c_int32),
                ("ks_level", C.c_int32), ("pbs_base_log", C.c_int32), ("pbs_level", C.c_int32),
                ("ring", C.c_int32), ("lwe_sigma", C.c_double), ("glwe_sigma", C.c_double)]


class MatchStats(C.Structure):
    _fields_ = [("ct_ops", C.c_uint64), ("cache_hits", C.c_uint64), ("n_branches", C.c_uint64),
                ("pbs", C.c_uint64), ("blind_rotations", C.c_uint64), ("levels", C.c_uint64), ("max_level_width", C.c_uint64),
                ("host_ms", C.c_double), ("device_ms", C.c_double), ("br_kernel_ms", C.c_double),
                ("ks_kernel_ms", C.c_double), ("br_launches", C.c_uint64), ("br_gates", C.c_uint64),
                ("plan_cached", C.c_uint64)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class PlainResult(C.Structure):
    _fields_ = [("ct_ops", C.c_uint64), ("cache_hits", C.c_uint64), ("n_branches", C.c_uint64),
                ("pbs", C.c_uint64), ("levels", C.c_uint64), ("max_level_width", C.c_uint64),
                ("result_recorded", C.c_int32), ("result_lowered", C.c_int32)]


GATE_LUT, GATE_SIGN = 0, 1


class Gate(C.Structure):
    """fr_gate: offset in units of Delta/2; kind GATE_LUT or GATE_SIGN."""
    _fields_ = [("n_in", C.c_int32), ("offset", C.c_int32), ("kind", C.c_int32), ("in_", C.c_uint32 * 16),
                ("in_block", C.c_int8 * 16), ("in_w", C.c_int8 * 16), ("lut", C.c_uint8 * 16),
                ("out", C.c_uint32)]


class FrJob(C.Structure):
    """fr_job: one rotation job of a match schedule (fr_schedule_match)."""
    _fields_ = [("n_in", C.c_int32), ("offset", C.c_int32), ("in_ref", C.c_int32 * 16), ("in_w", C.c_int32 * 16),
                ("n_out", C.c_int32), ("kind", C.c_int32), ("out_gate", C.c_int32 * 8), ("lut", (C.c_uint8 * 16) * 8)]


JOB_MULTI, JOB_DIRECT, JOB_SIGN = 0, 1, 2

u64p = C.POINTER(C.c_uint64)
_lib = None

# every exported symbol of include/fheregex.h, with (restype, argtypes)
_SIGS = {
    "fr_ctx_create": (C.c_int, [C.POINTER(Params), C.c_int, C.POINTER(C.c_void_p)]),
    "fr_ctx_destroy": (C.c_int, [C.c_void_p]),
    "fr_last_error": (C.c_char_p, []),
    "fr_default_params": (C.c_int, [C.POINTER(Params)]),
    "fr_load_client_key": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "fr_gen_client_key": (C.c_int, [C.c_void_p, C.c_uint64]),
    "fr_serialize_client_key": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "fr_gen_server_key": (C.c_int, [C.c_void_p, C.c_uint64]),
    "fr_set_keygen": (C.c_int, [C.c_void_p, C.c_int32]),
    "fr_export_server_key": (C.c_int, [C.c_void_p, u64p, C.c_size_t, u64p, C.c_size_t]),
    "fr_server_key_sizes": (C.c_int, [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "fr_load_server_key": (C.c_int, [C.c_void_p, u64p, C.c_size_t, u64p, C.c_size_t]),
    "fr_encrypt_str": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, C.c_uint64, u64p]),
    "fr_encrypt_blocks": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t, C.c_uint64, C.c_uint64, u64p]),
    "fr_decrypt_radix": (C.c_int, [C.c_void_p, u64p, u64p]),
    "fr_decode_block": (C.c_int, [C.c_void_p, u64p, C.POINTER(C.c_uint32)]),
    "fr_upload_radix": (C.c_int, [C.c_void_p, u64p, C.c_size_t, C.POINTER(C.c_uint32)]),
    "fr_upload_bool": (C.c_int, [C.c_void_p, u64p, C.c_size_t, C.POINTER(C.c_uint32)]),
    "fr_encrypt_upload_str": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, C.c_uint64, C.POINTER(C.c_uint32)]),
    "fr_radix_serialize": (C.c_int, [C.c_void_p, u64p, C.c_size_t, C.c_uint64, C.c_char_p, C.c_size_t,
                                     C.POINTER(C.c_size_t)]),
    "fr_radix_deserialize": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, u64p, C.c_size_t,
                                       C.POINTER(C.c_size_t)]),
    "fr_download_radix": (C.c_int, [C.c_void_p, C.c_uint32, u64p]),
    "fr_release": (C.c_int, [C.c_void_p, C.c_uint32]),
    "fr_trivial": (C.c_int, [C.c_void_p, C.c_uint8, C.POINTER(C.c_uint32)]),
    "fr_eq_const": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint8, C.POINTER(C.c_uint32)]),
    "fr_gt_const": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint8, C.POINTER(C.c_uint32)]),
    "fr_le_const": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint8, C.POINTER(C.c_uint32)]),
    "fr_and": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    "fr_or": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    "fr_not": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "fr_or_many": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_uint32)]),
    "fr_run_gates": (C.c_int, [C.c_void_p, C.POINTER(Gate), C.c_size_t]),
    "fr_has_match": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.c_char_p, C.POINTER(C.c_uint32),
                               C.POINTER(MatchStats)]),
    "fr_has_match_range": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.c_char_p, C.c_size_t,
                                     C.c_size_t, C.POINTER(C.c_uint32), C.POINTER(MatchStats)]),
    "fr_has_match_parts": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.c_char_p, C.c_size_t,
                                     C.c_size_t, C.c_size_t, C.POINTER(C.c_uint32), C.POINTER(C.c_size_t),
                                     C.POINTER(MatchStats)]),
    "fr_plain_match_parts": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t, C.c_int32,
                                       C.c_int32, C.c_int32, C.c_size_t, C.POINTER(PlainResult),
                                       C.POINTER(C.c_int32), C.POINTER(C.c_size_t)]),
    "fr_schedule_match_parts": (C.c_int, [C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t, C.c_int32, C.c_int32,
                                          C.c_int32, C.c_int32, C.c_size_t, C.POINTER(FrJob), C.c_size_t,
                                          C.POINTER(C.c_size_t), C.POINTER(C.c_uint32), C.c_size_t,
                                          C.POINTER(C.c_size_t), C.POINTER(C.c_int32), C.POINTER(C.c_size_t)]),
    "fr_debug_enumeration_cost": (C.c_int, [C.c_char_p, C.c_int32, C.c_size_t, C.c_size_t, C.c_size_t, C.c_uint64,
                                            C.c_uint64, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_uint64),
                                            C.POINTER(C.c_uint64)]),
    "fr_parse": (C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t]),
    "fr_set_plan_cache": (C.c_int, [C.c_void_p, C.c_size_t]),
    "fr_set_plan_cache_slots": (C.c_int, [C.c_void_p, C.c_size_t]),
    "fr_set_async": (C.c_int, [C.c_void_p, C.c_int32]),
    "fr_set_lanes": (C.c_int, [C.c_void_p, C.c_int32]),
    "fr_plan_cache_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "fr_has_match_batch": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.c_size_t, C.c_char_p,
                                     C.POINTER(C.c_uint32), C.POINTER(MatchStats)]),
    "fr_set_engine": (C.c_int, [C.c_void_p, C.c_int32]),
    "fr_set_grammar": (C.c_int, [C.c_void_p, C.c_int32]),
    "fr_parse_ex": (C.c_int, [C.c_char_p, C.c_int32, C.c_char_p, C.c_size_t]),
    "fr_plain_match_g": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t, C.c_int32, C.c_int32,
                                   C.c_int32, C.POINTER(PlainResult)]),
    "fr_plain_match_ex": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t, C.c_int32, C.c_int32,
                                    C.POINTER(PlainResult)]),
    "fr_plain_match": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t, C.c_int32,
                                 C.POINTER(PlainResult)]),
    "fr_set_lowering": (C.c_int, [C.c_void_p, C.c_int32]),
    "fr_set_profiling": (C.c_int, [C.c_void_p, C.c_int32]),
    "fr_set_multi_value": (C.c_int, [C.c_void_p, C.c_int32]),
    "fr_dev_blind_rotate_multi": (C.c_int, [C.c_void_p, u64p, C.POINTER(C.c_uint8), C.c_int32, C.c_int32, u64p]),
    "fr_dev_keyswitch": (C.c_int, [C.c_void_p, u64p, C.c_size_t, u64p]),
    "fr_dev_blind_rotate": (C.c_int, [C.c_void_p, u64p, C.POINTER(C.c_uint8), C.c_size_t, u64p]),
    "fr_dev_ring_mul": (C.c_int, [C.c_void_p, u64p, u64p, C.c_size_t, u64p]),
    "fr_dev_bench_pbs": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.c_int32,
                                   C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "fr_device_info": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "fr_debug_scalar": (C.c_uint64, [C.c_int32, C.c_uint64, C.c_uint64]),
    "fr_export_bool_device": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.c_void_p]),
    "fr_export_bool_device_async": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.c_void_p]),
    "fr_stream": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "fr_import_bool_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint32)]),
    "fr_device_timers": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint64)]),
    "fr_device_timers_latency": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                           C.POINTER(C.c_uint64)]),
    "fr_device_timers_pair": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64)]),
    "fr_shard_plan": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t,
                                C.POINTER(C.c_void_p), C.POINTER(MatchStats)]),
    "fr_shard_levels": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "fr_shard_jobs": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "fr_shard_outputs": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    "fr_shard_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]),
    "fr_shard_export": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]),
    "fr_shard_import": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]),
    "fr_shard_finish": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(MatchStats)]),
    "fr_shard_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "fr_schedule_match": (C.c_int, [C.c_size_t, C.c_char_p, C.c_size_t, C.c_size_t, C.c_int32, C.c_int32, C.c_int32,
                                    C.c_int32, C.POINTER(FrJob), C.c_size_t, C.POINTER(C.c_size_t),
                                    C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_int32)]),
}


def lib():
    """Load the in-tree libfheregex.so (fails loudly if it was not built).

    A process that also uses torch on the GPU imports torch first: the torch wheel
    bundles its own HIP runtime with the soname of /opt/rocm's, so loaded first it is the
    one runtime this library binds to; loaded second, torch finds no device."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C {HERE}` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc: int):
    if rc == FR_OK:
        return
    msg = lib().fr_last_error().decode(errors="replace")
    cls = {ERR_PARSE: ParseError, ERR_REF_PANIC: ReferencePanic, ERR_NO_DEVICE: NoDevice}.get(rc, FheRegexError)
    if rc == ERR_NON_ASCII:
        raise ValueError(msg)
    raise cls(rc, msg)


def _p(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u64p)


RING_RNS, RING_FFT = 0, 1  # fheregex.h FR_RING_*


def default_params(k: Optional[int] = None, N: Optional[int] = None, ring: Optional[int] = None) -> Params:
    p = Params()
    _check(lib().fr_default_params(C.byref(p)))
    if k is not None:
        p.k = k
    if N is not None:
        p.N = N
    if ring is not None:
        p.ring = ring
    elif (p.k, p.N) not in ((1, 2048), (2, 1024)):
        p.ring = RING_RNS  # the FFT ring is built for k = 1, N = 2048 and k = 2, N = 1024
    return p


def parse(pattern: str, grammar: int = GRAMMAR_REFERENCE) -> str:
    """Canonical AST string (parser.rs:146-185; GRAMMAR_EXT: the opt-in class extension)."""
    size = 1 << 16
    while True:
        buf = C.create_string_buffer(size)
        rc = lib().fr_parse_ex(pattern.encode("latin-1"), grammar, buf, len(buf))
        if rc == ERR_INVALID and size < (1 << 28) and b"buffer too small" in lib().fr_last_error():
            size <<= 2
            continue
        _check(rc)
        return buf.value.decode()


def plain_match(content: bytes | str, pattern: str, lowering: int = LOWER_THRESHOLD,
                start_lo: int = 0, start_hi: Optional[int] = None, engine: int = ENGINE_ENUMERATE,
                grammar: int = GRAMMAR_REFERENCE) -> PlainResult:
    """Host-only symbolic run: reference counters + plaintext result of the
    recorded circuit and of the lowered PBS program."""
    if isinstance(content, str):
        content = content.encode("latin-1")
    hi = len(content) if start_hi is None else start_hi
    r = PlainResult()
    _check(lib().fr_plain_match_g(content, len(content), pattern.encode("latin-1"), start_lo, hi, lowering, engine,
                                  grammar, C.byref(r)))
    return r


COST_COUNTED, COST_PANIC, COST_MEMORY = 0, 1, 2


def enumeration_cost(pattern: str, n_chars: int, start_lo: int = 0, start_hi: Optional[int] = None,
                     cap: int = 1 << 22, enumerate: bool = False, grammar: int = GRAMMAR_REFERENCE,
                     mem_bytes: int = 0, with_outcome: bool = False):
    """(counted, enumerated): the reference enumeration's variant count from the AST
    (None without a count: where it would panic, or past the counter's memo bound
    mem_bytes, 0 = AUTO's) and, if asked, by enumerating; both saturate at cap + 1.
    with_outcome: (outcome, counted, enumerated), outcome one of COST_*."""
    hi = n_chars if start_hi is None else start_hi
    o, c, e = C.c_int32(), C.c_uint64(), C.c_uint64()
    _check(lib().fr_debug_enumeration_cost(pattern.encode("latin-1"), grammar, n_chars, start_lo, hi, cap, mem_bytes,
                                           int(enumerate), C.byref(o), C.byref(c), C.byref(e)))
    counted = c.value if o.value == COST_COUNTED else None
    enumerated = e.value if enumerate else None
    return (o.value, counted, enumerated) if with_outcome else (counted, enumerated)


def plain_match_parts(content: bytes | str, pattern: str, start_lo: int, start_hi: int, max_parts: int,
                      lowering: int = LOWER_THRESHOLD, engine: int = ENGINE_ENUMERATE,
                      grammar: int = GRAMMAR_REFERENCE):
    """Host-only run of fr_has_match_parts' program: (PlainResult with result_lowered =
    the OR of the parts, [plaintext value of each part])"""
    if isinstance(content, str):
        content = content.encode("latin-1")
    r = PlainResult()
    vals = (C.c_int32 * max_parts)()
    n = C.c_size_t()
    _check(lib().fr_plain_match_parts(content, len(content), pattern.encode("latin-1"), start_lo, start_hi, lowering,
                                      engine, grammar, max_parts, C.byref(r), vals, C.byref(n)))
    return r, list(vals)[:n.value]


class Context:
    """One fr_ctx: params, keys, device arena.  device=-1: host-only."""

    def __init__(self, device: int = 0, params: Optional[Params] = None):
        self.params = params if params is not None else default_params()
        h = C.c_void_p()
        _check(lib().fr_ctx_create(C.byref(self.params), device, C.byref(h)))
        self.h = h
        self.device = device
        self.big = self.params.k * self.params.N
        self.lwe_len = self.big + 1

    def close(self):
        if getattr(self, "h", None):
            lib().fr_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> str:
        buf = C.create_string_buffer(256)
        _check(lib().fr_device_info(self.h, buf, 256))
        return buf.value.decode()

    # keys
    def load_client_key(self, blob: bytes):
        _check(lib().fr_load_client_key(self.h, blob, len(blob)))

    def gen_client_key(self, seed: int):
        """gen_keys_radix(&PARAM_MESSAGE_2_CARRY_2, 4) (ciphertext.rs:44): a fresh
        uniform binary client key, reproducible from `seed`."""
        _check(lib().fr_gen_client_key(self.h, seed & 0xFFFFFFFFFFFFFFFF))

    def serialize_client_key(self) -> bytes:
        """bincode RadixClientKey (engine.rs:238-246 generate_test_keys): the layout
        load_client_key reads; a loaded key comes back byte for byte."""
        n = C.c_size_t()
        _check(lib().fr_serialize_client_key(self.h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        _check(lib().fr_serialize_client_key(self.h, buf, n.value, C.byref(n)))
        return buf.raw

    def gen_server_key(self, seed: int):
        """ServerKey::new (engine.rs:252): on the GPU for the FFT ring (KEYGEN_AUTO),
        else on the host; both give the same key bit for bit."""
        _check(lib().fr_gen_server_key(self.h, seed))

    def set_keygen(self, where: int):
        """KEYGEN_AUTO (device when present, FFT ring), KEYGEN_HOST or KEYGEN_DEVICE."""
        _check(lib().fr_set_keygen(self.h, where))

    def export_server_key(self):
        a, b = C.c_size_t(), C.c_size_t()
        _check(lib().fr_server_key_sizes(self.h, C.byref(a), C.byref(b)))
        ksk = np.zeros(a.value, dtype=np.uint64)
        bsk = np.zeros(b.value, dtype=np.uint64)
        _check(lib().fr_export_server_key(self.h, _p(ksk), len(ksk), _p(bsk), len(bsk)))
        return ksk, bsk

    def load_server_key(self, ksk: np.ndarray, bsk: np.ndarray):
        """install an exported server key (export_server_key's arrays): a server context
        holding only sk, as has_match(sk, ...) takes it (engine.rs:8); no client key needed"""
        k = np.ascontiguousarray(ksk, dtype=np.uint64)
        b = np.ascontiguousarray(bsk, dtype=np.uint64)
        _check(lib().fr_load_server_key(self.h, _p(k), len(k), _p(b), len(b)))

    def set_lowering(self, mode: int):
        _check(lib().fr_set_lowering(self.h, mode))

    def set_engine(self, engine: int):
        """ENGINE_AUTO (default), ENGINE_ENUMERATE (the reference's variant
        enumeration) or ENGINE_MERGED (state merging; same decrypted result)."""
        _check(lib().fr_set_engine(self.h, engine))

    def set_grammar(self, grammar: int):
        """GRAMMAR_REFERENCE (default: parser.rs exactly) or GRAMMAR_EXT (also
        bare digits and mixed bracket classes such as [a-z0-9]; beyond the reference)."""
        _check(lib().fr_set_grammar(self.h, grammar))

    def set_multi_value(self, on: bool):
        _check(lib().fr_set_multi_value(self.h, int(on)))

    def set_plan_cache(self, capacity: int):
        """Plans kept for repeat has_match calls (0: off, frees the cached plans)."""
        _check(lib().fr_set_plan_cache(self.h, capacity))

    def set_async(self, on: bool):
        """has_match returns once its launches are enqueued (default) or blocks (False)."""
        _check(lib().fr_set_async(self.h, int(on)))

    def set_lanes(self, n: int):
        """fr_set_lanes: consecutive asynchronous matches round-robin over n streams of this
        context (one key, a plan copy per lane); every other call waits for them device-side."""
        _check(lib().fr_set_lanes(self.h, int(n)))

    def set_plan_cache_slots(self, max_slots: int):
        """Bound on the intermediate arena slots held by all cached plans."""
        _check(lib().fr_set_plan_cache_slots(self.h, max_slots))

    def plan_cache_stats(self):
        v = [C.c_uint64() for _ in range(4)]
        _check(lib().fr_plan_cache_stats(self.h, *[C.byref(x) for x in v]))
        return dict(zip(("entries", "slots", "hits", "misses"), (x.value for x in v)))

    def set_profiling(self, on):
        """0/False off, 1/True blind-rotation timers, 2 also keyswitch timers (fr_set_profiling)."""
        _check(lib().fr_set_profiling(self.h, int(on)))

    # client side
    def encrypt_str(self, s: bytes | str, seed: int) -> np.ndarray:
        if isinstance(s, str):
            s = s.encode("latin-1")
        out = np.zeros((len(s), 4, self.lwe_len), dtype=np.uint64)
        _check(lib().fr_encrypt_str(self.h, s, len(s), seed, _p(out)))
        return out

    def encrypt_blocks(self, msgs, seed: int, first_block: int = 0) -> np.ndarray:
        m = np.ascontiguousarray(np.asarray(msgs, dtype=np.uint8))
        out = np.zeros((len(m), self.lwe_len), dtype=np.uint64)
        _check(lib().fr_encrypt_blocks(self.h, m.ctypes.data_as(C.POINTER(C.c_uint8)), len(m), seed, first_block, _p(out)))
        return out

    def decrypt_radix(self, blocks: np.ndarray) -> int:
        b = np.ascontiguousarray(blocks, dtype=np.uint64)
        v = C.c_uint64()
        _check(lib().fr_decrypt_radix(self.h, _p(b), C.byref(v)))
        return v.value

    def decode_block(self, lwe: np.ndarray) -> int:
        b = np.ascontiguousarray(lwe, dtype=np.uint64)
        v = C.c_uint32()
        _check(lib().fr_decode_block(self.h, _p(b), C.byref(v)))
        return v.value

    # arena
    def upload_radix(self, blocks: np.ndarray) -> List[int]:
        b = np.ascontiguousarray(blocks.reshape(-1, 4, self.lwe_len), dtype=np.uint64)
        out = (C.c_uint32 * b.shape[0])()
        _check(lib().fr_upload_radix(self.h, _p(b), b.shape[0], out))
        return list(out)

    def encrypt_upload_str(self, s: bytes | str, seed: int) -> List[int]:
        """encrypt_str on the device into content handles (same words as encrypt_str)."""
        if isinstance(s, str):
            s = s.encode("latin-1")
        out = (C.c_uint32 * len(s))()
        _check(lib().fr_encrypt_upload_str(self.h, s, len(s), seed, out))
        return list(out)

    def serialize_radix(self, blocks: np.ndarray, degree: int = 3) -> bytes:
        """bincode RadixCiphertext (tfhe-rs 0.2 layout, [ext] unverified) of one radix (4 blocks)."""
        b = np.ascontiguousarray(blocks.reshape(-1, self.lwe_len), dtype=np.uint64)
        n = C.c_size_t()
        _check(lib().fr_radix_serialize(self.h, _p(b), b.shape[0], degree, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        _check(lib().fr_radix_serialize(self.h, _p(b), b.shape[0], degree, buf, n.value, C.byref(n)))
        return buf.raw

    def deserialize_radix(self, data: bytes) -> np.ndarray:
        n = C.c_size_t()
        _check(lib().fr_radix_deserialize(self.h, data, len(data), None, 0, C.byref(n)))
        out = np.zeros((n.value, self.lwe_len), dtype=np.uint64)
        _check(lib().fr_radix_deserialize(self.h, data, len(data), _p(out), n.value, C.byref(n)))
        return out

    def upload_bool(self, lwes: np.ndarray) -> List[int]:
        b = np.ascontiguousarray(lwes.reshape(-1, self.lwe_len), dtype=np.uint64)
        out = (C.c_uint32 * b.shape[0])()
        _check(lib().fr_upload_bool(self.h, _p(b), b.shape[0], out))
        return list(out)

    def download_radix(self, h: int) -> np.ndarray:
        out = np.zeros((4, self.lwe_len), dtype=np.uint64)
        _check(lib().fr_download_radix(self.h, h, _p(out)))
        return out

    def release(self, h: int):
        _check(lib().fr_release(self.h, h))

    def trivial(self, v: int) -> int:
        out = C.c_uint32()
        _check(lib().fr_trivial(self.h, v, C.byref(out)))
        return out.value

    # eager ops (the smart_* replacements)
    def _op1c(self, fn, a, c):
        out = C.c_uint32()
        _check(fn(self.h, a, c, C.byref(out)))
        return out.value

    def eq_const(self, a, c): return self._op1c(lib().fr_eq_const, a, c)
    def gt_const(self, a, c): return self._op1c(lib().fr_gt_const, a, c)
    def le_const(self, a, c): return self._op1c(lib().fr_le_const, a, c)
    def and_(self, a, b): return self._op1c(lib().fr_and, a, b)
    def or_(self, a, b): return self._op1c(lib().fr_or, a, b)

    def not_(self, a):
        out = C.c_uint32()
        _check(lib().fr_not(self.h, a, C.byref(out)))
        return out.value

    def or_many(self, hs: Sequence[int]) -> int:
        arr = (C.c_uint32 * len(hs))(*hs)
        out = C.c_uint32()
        _check(lib().fr_or_many(self.h, arr, len(hs), C.byref(out)))
        return out.value

    def or_each(self, groups: Sequence[Sequence[int]]) -> List[int]:
        """one OR per group of <= 16 booleans, all groups in one launch (fr_run_gates:
        independent sign gates, the threshold OR of fr_or_many): the final bitor of
        many start-sharded matches at once"""
        gates = []
        for grp in groups:
            if not 1 <= len(grp) <= 16:
                raise ValueError("or_each: 1..16 booleans per group")
            g = Gate()
            g.n_in, g.offset, g.kind = len(grp), -1, GATE_SIGN
            for q, h in enumerate(grp):
                g.in_[q], g.in_block[q], g.in_w[q] = h, 0, 1
            gates.append(g)
        return self.run_gates(gates) if gates else []

    def run_gates(self, gates: Sequence[Gate]) -> List[int]:
        arr = (Gate * len(gates))(*gates)
        _check(lib().fr_run_gates(self.h, arr, len(gates)))
        return [g.out for g in arr]

    def has_match(self, content: Sequence[int], pattern: str, start_lo: Optional[int] = None,
                  start_hi: Optional[int] = None):
        """engine.rs:8-42 over content handles (a sequence, or a uint32 numpy array: no copy)"""
        if isinstance(content, np.ndarray):
            content = np.ascontiguousarray(content, dtype=np.uint32)
            arr = content.ctypes.data_as(C.POINTER(C.c_uint32))
        else:
            arr = (C.c_uint32 * len(content))(*content)
        out = C.c_uint32()
        st = MatchStats()
        if start_lo is None and start_hi is None:
            _check(lib().fr_has_match(self.h, arr, len(content), pattern.encode("latin-1"), C.byref(out), C.byref(st)))
        else:
            lo = 0 if start_lo is None else start_lo
            hi = len(content) if start_hi is None else start_hi
            _check(lib().fr_has_match_range(self.h, arr, len(content), pattern.encode("latin-1"), lo, hi,
                                            C.byref(out), C.byref(st)))
        return out.value, st

    def has_match_parts(self, content: Sequence[int], pattern: str, start_lo: int, start_hi: int, max_parts: int):
        """fr_has_match_parts: ([<= max_parts boolean handles whose OR is the range's
        match], stats) -- a start shard's result for a caller-side OR over shards"""
        content = np.ascontiguousarray(content, dtype=np.uint32)
        arr = content.ctypes.data_as(C.POINTER(C.c_uint32))
        out = (C.c_uint32 * max_parts)()
        n = C.c_size_t()
        st = MatchStats()
        _check(lib().fr_has_match_parts(self.h, arr, len(content), pattern.encode("latin-1"), start_lo, start_hi,
                                        max_parts, out, C.byref(n), C.byref(st)))
        return list(out)[:n.value], st

    def has_match_batch(self, contents: Sequence[Sequence[int]], pattern: str):
        """M independent matches of one pattern over M equal-length contents in
        shared launches (fr_has_match_batch): ([out handle per match], stats)."""
        M = len(contents)
        n = len(contents[0]) if M else 0
        if any(len(c) != n for c in contents):
            raise ValueError("has_match_batch: contents must have one length")
        flat = [h for c in contents for h in c]
        arr = (C.c_uint32 * max(len(flat), 1))(*flat)
        out = (C.c_uint32 * max(M, 1))()
        st = MatchStats()
        _check(lib().fr_has_match_batch(self.h, arr, n, M, pattern.encode("latin-1"), out, C.byref(st)))
        return list(out)[:M], st

    def export_bool_device(self, hs: Sequence[int], dev_ptr: int):
        arr = (C.c_uint32 * len(hs))(*hs)
        _check(lib().fr_export_bool_device(self.h, arr, len(hs), C.c_void_p(dev_ptr)))

    def export_bool_device_async(self, hs: Sequence[int], dev_ptr: int):
        """stream-ordered export (no synchronisation): order other streams after it with
        an event on stream_ptr()"""
        arr = (C.c_uint32 * len(hs))(*hs)
        _check(lib().fr_export_bool_device_async(self.h, arr, len(hs), C.c_void_p(dev_ptr)))

    def stream_ptr(self) -> int:
        """the context's hipStream_t (for torch.cuda.ExternalStream)"""
        s = C.c_void_p()
        _check(lib().fr_stream(self.h, C.byref(s)))
        return s.value or 0

    def import_bool_device(self, dev_ptr: int, n: int) -> List[int]:
        out = (C.c_uint32 * n)()
        _check(lib().fr_import_bool_device(self.h, C.c_void_p(dev_ptr), n, out))
        return list(out)

    def device_timers(self):
        br, ks = C.c_double(), C.c_double()
        nl, ng = C.c_uint64(), C.c_uint64()
        _check(lib().fr_device_timers(self.h, C.byref(br), C.byref(ks), C.byref(nl), C.byref(ng)))
        lb, ll, lg = C.c_double(), C.c_uint64(), C.c_uint64()
        _check(lib().fr_device_timers_latency(self.h, C.byref(lb), C.byref(ll), C.byref(lg)))
        pb, pl, pg = C.c_double(), C.c_uint64(), C.c_uint64()
        _check(lib().fr_device_timers_pair(self.h, C.byref(pb), C.byref(pl), C.byref(pg)))
        return {"br_ms": br.value, "ks_ms": ks.value, "br_launches": nl.value, "br_gates": ng.value,
                "lat_br_ms": lb.value, "lat_launches": ll.value, "lat_gates": lg.value,
                "pair_br_ms": pb.value, "pair_launches": pl.value, "pair_gates": pg.value}

    # single-stage device entry points
    def dev_keyswitch(self, lwes: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(lwes.reshape(-1, self.lwe_len), dtype=np.uint64)
        out = np.zeros((a.shape[0], self.params.n + 1), dtype=np.uint64)
        _check(lib().fr_dev_keyswitch(self.h, _p(a), a.shape[0], _p(out)))
        return out

    def dev_blind_rotate(self, ks: np.ndarray, luts) -> np.ndarray:
        a = np.ascontiguousarray(ks.reshape(-1, self.params.n + 1), dtype=np.uint64)
        l = np.ascontiguousarray(np.asarray(luts, dtype=np.uint8).reshape(a.shape[0], 16))
        out = np.zeros((a.shape[0], self.lwe_len), dtype=np.uint64)
        _check(lib().fr_dev_blind_rotate(self.h, _p(a), l.ctypes.data_as(C.POINTER(C.c_uint8)), a.shape[0], _p(out)))
        return out

    def dev_blind_rotate_multi(self, ks: np.ndarray, luts, direct: bool = False) -> np.ndarray:
        a = np.ascontiguousarray(ks.reshape(self.params.n + 1), dtype=np.uint64)
        l = np.ascontiguousarray(np.asarray(luts, dtype=np.uint8).reshape(-1, 16))
        out = np.zeros((l.shape[0], self.lwe_len), dtype=np.uint64)
        _check(lib().fr_dev_blind_rotate_multi(self.h, _p(a), l.ctypes.data_as(C.POINTER(C.c_uint8)), l.shape[0],
                                               int(direct), _p(out)))
        return out

    def dev_ring_mul(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a.reshape(-1, self.params.N), dtype=np.uint64)
        b = np.ascontiguousarray(b.reshape(-1, self.params.N), dtype=np.uint64)
        out = np.zeros_like(a)
        _check(lib().fr_dev_ring_mul(self.h, _p(a), _p(b), a.shape[0], _p(out)))
        return out

    def dev_bench_pbs(self, handles: Sequence[int], iters: int):
        arr = (C.c_uint32 * len(handles))(*handles)
        br, tot = C.c_double(), C.c_double()
        _check(lib().fr_dev_bench_pbs(self.h, arr, len(handles), iters, C.byref(br), C.byref(tot)))
        return br.value, tot.value


# ------------------------------------------------------------- reference API
@dataclass
class ClientKey:
    ctx: Context

    def encrypt_str(self, s: str, seed: int = 0) -> List[int]:
        """encrypt_str (ciphertext.rs:32-40) + upload: one radix handle per char."""
        if any(ord(ch) > 127 for ch in s):
            raise ValueError("content contains non-ascii characters")
        return self.ctx.upload_radix(self.ctx.encrypt_str(s, seed))

    def decrypt(self, ct: int) -> int:
        return self.ctx.decrypt_radix(self.ctx.download_radix(ct))

    def serialize(self) -> bytes:
        """bincode::serialize of the RadixClientKey (engine.rs:238-246)."""
        return self.ctx.serialize_client_key()


@dataclass
class ServerKey:
    ctx: Context

    def create_trivial_radix(self, msg: int) -> int:
        return self.ctx.trivial(msg)

    def save(self, path: str):
        """the server key as an .npz of its (ksk, bsk) arrays (fr_export_server_key's layout)"""
        ksk, bsk = self.ctx.export_server_key()
        np.savez(path, ksk=ksk, bsk=bsk)

    @staticmethod
    def load(path: str, device: int = 0, params: Optional[Params] = None) -> "ServerKey":
        """a server context holding only this server key (fr_load_server_key; no client key)"""
        ctx = Context(device, params)
        with np.load(path, allow_pickle=False) as z:
            ctx.load_server_key(z["ksk"], z["bsk"])
        return ServerKey(ctx)


def gen_keys(client_key_blob: Optional[bytes] = None, seed: int = 0, device: int = 0,
             params: Optional[Params] = None, client_seed: Optional[int] = None):
    """gen_keys (ciphertext.rs:42-45): (client key, server key).

    Without a blob the client key is fresh (gen_keys_radix(&PARAM_MESSAGE_2_CARRY_2, 4),
    ciphertext.rs:44), drawn from `client_seed` (default: 64 bits of os.urandom, as the
    reference draws from the OS); with a blob it is that bincode key (read_test_keys,
    engine.rs:248-254).  The server key is derived deterministically from `seed`
    (ServerKey::new, engine.rs:252)."""
    ctx = Context(device, params)
    if client_key_blob is None:
        if client_seed is None:
            client_seed = int.from_bytes(os.urandom(8), "little")
        ctx.gen_client_key(client_seed)
    else:
        ctx.load_client_key(client_key_blob)
    ctx.gen_server_key(seed)
    return ClientKey(ctx), ServerKey(ctx)


def has_match(sk: ServerKey, content: Sequence[int], pattern: str) -> int:
    """engine.rs:8-42: returns the encrypted 0/1 result handle."""
    out, _ = sk.ctx.has_match(content, pattern)
    return out


def shard_starts(L: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous range [lo, hi) of start offsets owned by `rank`.

    The reference's driver ORs one branch set per start offset
    (engine.rs:22-35); offsets are independent, so ranks split them into
    contiguous ranges, evaluate their OR tree locally (fr_has_match_range) and
    a final OR over the gathered per-rank booleans gives the full result."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(L, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


# ------------------------------------------------------- one match across ranks
def job_slice(J: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous slice [a, b) of a level's J rotation jobs owned by `rank`
    (ceil(r J / world) boundaries: balanced, and rank 0 owns a lone job)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return -(-rank * J // world), -(-(rank + 1) * J // world)


def run_sharded(ex, world: int, rank: int, all_gather, times=None):
    """Level-sharded evaluation of one match plan (fheregex.h fr_shard_*):
    every level but the last is split into contiguous job slices, each rank runs
    its slice, and the slices' output LWEs are all-gathered so that every rank
    holds the level; rank 0 runs the last level.  `ex` is an executor (ShardPlan
    on the GPU, or a CPU evaluator in tests) with levels / jobs(l) /
    outputs(l, a, b) / run(l, a, b) / export(l, a, b, cap) -> buffer /
    import_(l, a, b, buffer); all_gather(buffer) returns every rank's buffer in
    rank order.  `times` (a dict) accumulates wall milliseconds per phase: slices
    (runs + exports, which wait for the device), gather, import, top.  Returns the
    number of gathered LWEs."""
    import time
    clock = time.perf_counter

    def tick(phase, t0):
        if times is not None:
            times[phase] = times.get(phase, 0.0) + (clock() - t0) * 1e3
        return clock()

    gathered = 0
    nl = ex.levels
    t = clock()
    for l in range(nl - 1):
        parts = [job_slice(ex.jobs(l), world, r) for r in range(world)]
        counts = [ex.outputs(l, a, b) for a, b in parts]
        a, b = parts[rank]
        if b > a:
            ex.run(l, a, b)
        send = ex.export(l, a, b, max(counts))
        t = tick("slices_ms", t)
        bufs = all_gather(send)
        t = tick("gather_ms", t)
        for r, (ar, br) in enumerate(parts):
            if r != rank and counts[r]:
                ex.import_(l, ar, br, bufs[r])
        t = tick("import_ms", t)
        gathered += sum(counts)
    if rank == 0 and nl:
        ex.run(nl - 1, 0, ex.jobs(nl - 1))
    tick("top_ms", t)
    return gathered


def _runs(idx) -> List[Tuple[int, int]]:
    """maximal contiguous [a, b) runs of a sorted index list"""
    out = []
    for i in idx:
        if out and out[-1][1] == i:
            out[-1] = (out[-1][0], i + 1)
        else:
            out.append((i, i + 1))
    return out


def closure_parts(S: "Schedule", world: int):
    """Dependency-closure sharding of one match schedule (fr_schedule_match).

    The top of the circuit (the last level, widened downwards while it is fed by
    too few jobs to split evenly over `world` ranks) runs on rank 0; the jobs that feed it (the frontier)
    are cut into `world` contiguous parts, and rank r runs the transitive closure
    of its part (every job its part depends on, level by level; a job two parts
    need runs on both ranks).  Only the frontier outputs travel, once, to rank 0.
    The regex circuit is local in the content (a start's branch reads the
    characters after it, engine.rs:45-214), so a contiguous part's closure is a
    contiguous window of each level and the duplicated work is the few jobs at
    the window edges.

    Returns (runs, frontier, top): runs[r][l] = [(a, b), ...] job runs of level l
    that rank r executes before the gather; frontier[r] = [(l, a, b), ...] the
    runs of rank r's frontier part, in gather order; top[l] = the runs rank 0
    executes after the gather."""
    nl = len(S.level_off) - 1
    level = []
    for l in range(nl):
        level += [l] * (S.level_off[l + 1] - S.level_off[l])
    prod = {}
    for gi, j in enumerate(S.jobs):
        for f in range(j.n_out):
            prod[j.out_gate[f]] = gi

    def producers(js):
        return {prod[S.jobs[gi].in_ref[q]] for gi in js for q in range(S.jobs[gi].n_in) if S.jobs[gi].in_ref[q] >= 0}

    def by_level(js):
        per = [[] for _ in range(nl)]
        for gi in sorted(js):
            per[level[gi]].append(gi - S.level_off[level[gi]])
        return per

    top = set(range(S.level_off[nl - 1], S.level_off[nl])) if nl else set()
    front = producers(top) - top
    # widen while some rank would get no part, or the parts are uneven and few
    while 0 < len(front) and (len(front) < world or (len(front) % world and len(front) < 4 * world)):
        wider = producers(top | front) - top - front
        if len(wider) <= len(front):
            break
        top |= front
        front = wider
    front = sorted(front)
    runs, frontier = [], []
    for r in range(world):
        a, b = job_slice(len(front), world, r)
        part = front[a:b]
        need, stack = set(), list(part)
        while stack:
            gi = stack.pop()
            if gi in need:
                continue
            need.add(gi)
            stack += list(producers([gi]))
        runs.append([_runs(x) for x in by_level(need)])
        frontier.append([(l, x, y) for l, xs in enumerate(by_level(part)) for x, y in _runs(xs)])
    return runs, frontier, [_runs(x) for x in by_level(top)]


def run_closure_sharded(ex, S: "Schedule", world: int, rank: int, all_gather, parts=None, times=None):
    """One match over `world` ranks by dependency-closure sharding (closure_parts):
    no exchange until the top of the circuit, then one all_gather of the frontier
    LWEs (device to device with torch_all_gather) and rank 0 runs the top.  `ex`
    is a run_sharded executor whose schedule is S; `parts` = closure_parts(S,
    world), computed once by a caller that repeats the match (it costs
    milliseconds of host time).  `times` (a dict) accumulates this rank's wall
    milliseconds per phase: closure (its jobs and the export of its frontier, which
    waits for the device), gather, top (imports and the top's launches; the top's
    device time lands in the caller's finish).  Returns the number of gathered LWEs."""
    import time

    import torch

    clock = time.perf_counter

    def tick(phase, t0):
        if times is not None:
            times[phase] = times.get(phase, 0.0) + (clock() - t0) * 1e3
        return clock()

    t = clock()
    nl = ex.levels
    if nl != len(S.level_off) - 1 or any(ex.jobs(l) != S.level_off[l + 1] - S.level_off[l] for l in range(nl)):
        raise ValueError("executor and schedule disagree")
    runs, frontier, top = parts if parts is not None else closure_parts(S, world)
    for l in range(nl):
        for a, b in runs[rank][l]:
            ex.run(l, a, b)
    sizes = [sum(ex.outputs(l, a, b) for l, a, b in frontier[r]) for r in range(world)]
    if max(sizes, default=0):
        parts = [ex.export(l, a, b, ex.outputs(l, a, b)).reshape(-1)[:ex.outputs(l, a, b) * ex.lwe_len]
                 for l, a, b in frontier[rank]]
        cap = max(sizes) * ex.lwe_len
        have = sum(p.numel() for p in parts)
        if have < cap:
            parts.append(torch.zeros(cap - have, dtype=torch.int64,
                                     device=parts[0].device if parts else ex.buffer_device()))
        send = torch.cat(parts).contiguous()
        t = tick("closure_ms", t)
        bufs = all_gather(send)
        t = tick("gather_ms", t)
        if rank == 0:
            for r in range(1, world):
                off = 0
                for l, a, b in frontier[r]:
                    n = ex.outputs(l, a, b) * ex.lwe_len
                    ex.import_(l, a, b, bufs[r][off:off + n])
                    off += n
    else:
        t = tick("closure_ms", t)
    if rank == 0:
        for l in range(nl):
            for a, b in top[l]:
                ex.run(l, a, b)
    tick("top_ms", t)
    return sum(sizes)


class ShardPlan:
    """fr_shard_* executor for run_sharded: a compiled, device-resident plan of one
    match; buffers are torch CUDA tensors (export / import go device to device)."""

    def __init__(self, ctx: Context, content: Sequence[int], pattern: str, start_lo: int = 0,
                 start_hi: Optional[int] = None):
        self.ctx = ctx
        arr = (C.c_uint32 * len(content))(*content)
        hi = len(content) if start_hi is None else start_hi
        h = C.c_void_p()
        self.stats = MatchStats()
        _check(lib().fr_shard_plan(ctx.h, arr, len(content), pattern.encode("latin-1"), start_lo, hi, C.byref(h),
                                   C.byref(self.stats)))
        self.h = h
        self.lwe_len = ctx.lwe_len
        n = C.c_uint32()
        _check(lib().fr_shard_levels(h, C.byref(n)))
        self.levels = n.value
        self._jobs = []
        for l in range(self.levels):
            _check(lib().fr_shard_jobs(h, l, C.byref(n)))
            self._jobs.append(n.value)

    def jobs(self, level: int) -> int:
        return self._jobs[level]

    def buffer_device(self):
        import torch
        return torch.device("cuda", self.ctx.device)

    def outputs(self, level: int, a: int, b: int) -> int:
        n = C.c_uint32()
        _check(lib().fr_shard_outputs(self.h, level, a, b, C.byref(n)))
        return n.value

    def run(self, level: int, a: int, b: int):
        _check(lib().fr_shard_run(self.ctx.h, self.h, level, a, b))

    def export(self, level: int, a: int, b: int, cap: int):
        import torch
        buf = torch.empty(max(cap, 1) * self.ctx.lwe_len, dtype=torch.int64, device=f"cuda:{self.ctx.device}")
        _check(lib().fr_shard_export(self.ctx.h, self.h, level, a, b, C.c_void_p(buf.data_ptr())))
        return buf

    def import_(self, level: int, a: int, b: int, buf):
        _check(lib().fr_shard_import(self.ctx.h, self.h, level, a, b, C.c_void_p(buf.data_ptr())))

    def finish(self) -> Tuple[int, MatchStats]:
        out = C.c_uint32()
        st = MatchStats()
        _check(lib().fr_shard_finish(self.ctx.h, self.h, C.byref(out), C.byref(st)))
        return out.value, st

    def free(self):
        if getattr(self, "h", None):
            _check(lib().fr_shard_free(self.ctx.h, self.h))
            self.h = None


def torch_all_gather(group=None):
    """all_gather for run_sharded over torch.distributed (RCCL on GPU tensors):
    the returned views of one gathered tensor are valid once this returns."""
    import torch
    import torch.distributed as dist

    staged = dist.get_backend(group) == "gloo"  # gloo rehearsal: device buffers go through the host

    def gather(buf):
        world = dist.get_world_size(group)
        src = buf.cpu() if staged and buf.is_cuda else buf
        out = torch.empty(world * src.numel(), dtype=src.dtype, device=src.device)
        dist.all_gather_into_tensor(out, src, group=group)
        if staged and buf.is_cuda:
            out = out.to(buf.device)
        if out.is_cuda:
            torch.cuda.synchronize(out.device)  # the library reads it on its own stream
        return list(out.view(world, -1))
    return gather


@dataclass
class Schedule:
    """fr_schedule_match: rotation jobs by level, without a device."""
    jobs: list
    level_off: List[int]
    out_gate: int
    out_w: int
    out_const: int
    n_gates: int
    parts: List[Tuple[int, int, int]] = None  # (out_gate, out_w, out_const) of each part


def schedule_match(n_chars: int, pattern: str, start_lo: int = 0, start_hi: Optional[int] = None,
                   lowering: int = LOWER_THRESHOLD, engine: int = ENGINE_AUTO, grammar: int = GRAMMAR_REFERENCE,
                   multi_value: bool = True, max_parts: int = 1) -> Schedule:
    """max_parts > 1: fr_has_match_parts' schedule (Schedule.parts; out_* = part 0)"""
    hi = n_chars if start_hi is None else start_hi
    nj, nl, npart = C.c_size_t(), C.c_size_t(), C.c_size_t()
    outs3 = (C.c_int32 * (3 * max_parts))()
    pat = pattern.encode("latin-1")
    args = (n_chars, pat, start_lo, hi, lowering, engine, grammar, int(multi_value), max_parts)
    _check(lib().fr_schedule_match_parts(*args, None, 0, C.byref(nj), None, 0, C.byref(nl), outs3, C.byref(npart)))
    jobs = (FrJob * max(nj.value, 1))()
    off = (C.c_uint32 * (nl.value + 1))()
    _check(lib().fr_schedule_match_parts(*args, jobs, len(jobs), C.byref(nj), off, len(off), C.byref(nl), outs3,
                                         C.byref(npart)))
    n_gates = 1 + max([max(j.out_gate[f] for f in range(j.n_out)) for j in jobs[:nj.value]] or [-1])
    parts = [(outs3[3 * j], outs3[3 * j + 1], outs3[3 * j + 2]) for j in range(npart.value)]
    return Schedule(list(jobs[:nj.value]), list(off), parts[0][0], parts[0][1], parts[0][2], n_gates, parts)


def content_window(n_chars: int, pattern: str, start_lo: int, start_hi: int, lowering: int = LOWER_THRESHOLD,
                   engine: int = ENGINE_AUTO, grammar: int = GRAMMAR_REFERENCE) -> Tuple[int, int]:
    """[wlo, whi): the content positions the circuit of starts [start_lo, start_hi)
    reads, from its lowered schedule (a start's branch reads the characters after
    it, engine.rs:45-214): a start-offset shard needs only this window of the
    content.  (lo, lo) when the circuit reads no content."""
    S = schedule_match(n_chars, pattern, start_lo, start_hi, lowering=lowering, engine=engine, grammar=grammar)
    pos = [(-1 - j.in_ref[q]) // 4 for j in S.jobs for q in range(j.n_in) if j.in_ref[q] < 0]
    return (min(pos), max(pos) + 1) if pos else (start_lo, start_lo)


def header_symbols() -> List[str]:
    import re
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(fr_[a-z_]+)\s*\(", txt)) - {"fr_ctx", "FR_GATE_REF"})
