"""ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product; only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this file.

Plaintext CPU restatement of the reference's regex layer (RKlompUU/fhe-regex):

* ``parse``         — src/regex/parser.rs:146-351 (combine 4.6.6 grammar, modelled
                      with combine's commit/backtrack rules: a parser that fails
                      after consuming input is a *committed* error that ``choice``,
                      ``many`` and ``optional`` propagate; ``attempt`` turns it back
                      into an empty error).
* ``case_insensitive`` — src/regex/parser.rs:44-81.
* ``build_branches`` — src/regex/engine.rs:45-214 (list-monad variant enumerator).
* ``has_match``     — src/regex/engine.rs:8-42 (left fold of ct_or over branches).
* ``Execution``     — src/regex/execution.rs:8-223 (structural op-cache keys,
                      constant short-circuits, ct_ops / cache_hits counters).

Ciphertexts are replaced by their plaintext radix values (u8) so the result is
the reference's *decrypted* result.  Keys are hash-consed into integer ids so
that structural equality of ``Executed`` trees is id equality (the reference
hashes whole trees; the counts are identical).

Grammar extension (beyond the reference, ``ext=True``; mirrors the product's
FR_GRAMMAR_EXT): bare digits are characters, and a bracket whose reference
parse fails is re-read as a class of letters, digits, escapes and inclusive
ranges (``Class(lo-hi,...)``).  Patterns the reference accepts keep their AST.
Parity of the extension is against this restatement alone (the reference
returns Err for these patterns).

Reference panics (``parse_digits("")`` at parser.rs:349-351, ``Seq{[]}``
indexing at engine.rs:189-190) are raised as ``ReferencePanic``.

Parity pin: tests/golden/parser_vectors.json (the 49 cases of
src/regex/parser.rs:358-678) and tests/golden/engine_vectors.json (the 25 cases
of src/regex/engine.rs:256-280 plus SURVEY Appendix B op counts).
"""
from __future__ import annotations

import sys
from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

sys.setrecursionlimit(100000)


class ParseError(Exception):
    """Reference returns ``Err`` (anyhow) from ``parse``."""


class ReferencePanic(Exception):
    """The reference would panic (Rust unwrap / index out of bounds)."""


# --------------------------------------------------------------------------
# AST.  Canonical string form (shared with the C++ product's fr_parse):
#   SOF | EOF | Any | Char(c) | Between(f,t) | Range(c,...) | Not(x)
#   | Either(l,r) | Optional(x) | Repeated(x,lo,hi) (None -> _) | Seq(x,...)
# --------------------------------------------------------------------------

@dataclass(frozen=True)
class Node:
    kind: str
    c: int = 0
    f: int = 0
    t: int = 0
    cs: Tuple[int, ...] = ()
    a: Optional["Node"] = None
    b: Optional["Node"] = None
    lo: Optional[int] = None
    hi: Optional[int] = None
    xs: Tuple["Node", ...] = ()

    def __str__(self) -> str:  # canonical form
        k = self.kind
        if k in ("SOF", "EOF", "Any"):
            return k
        if k == "Char":
            return f"Char({self.c})"
        if k == "Between":
            return f"Between({self.f},{self.t})"
        if k == "Range":
            return "Range(" + ",".join(str(c) for c in self.cs) + ")"
        if k == "Not":
            return f"Not({self.a})"
        if k == "Either":
            return f"Either({self.a},{self.b})"
        if k == "Optional":
            return f"Optional({self.a})"
        if k == "Repeated":
            lo = "_" if self.lo is None else str(self.lo)
            hi = "_" if self.hi is None else str(self.hi)
            return f"Repeated({self.a},{lo},{hi})"
        if k == "Seq":
            return "Seq(" + ",".join(str(x) for x in self.xs) + ")"
        if k == "Class":
            return "Class(" + ",".join(f"{self.cs[i]}-{self.cs[i + 1]}" for i in range(0, len(self.cs), 2)) + ")"
        raise ValueError(k)


def case_insensitive(n: Node) -> Node:
    """parser.rs:44-81: only Char is folded; Range/Between/AnyChar are not."""
    k = n.kind
    if k == "Char":
        c = n.c
        if 97 <= c <= 122:
            return Node("Range", cs=(c, c - 32))
        if 65 <= c <= 90:
            return Node("Range", cs=(c, c + 32))
        return Node("Range", cs=(c,))
    if k == "Not":
        return Node("Not", a=case_insensitive(n.a))
    if k == "Either":
        return Node("Either", a=case_insensitive(n.a), b=case_insensitive(n.b))
    if k == "Optional":
        return Node("Optional", a=case_insensitive(n.a))
    if k == "Repeated":
        return Node("Repeated", a=case_insensitive(n.a), lo=n.lo, hi=n.hi)
    if k == "Seq":
        return Node("Seq", xs=tuple(case_insensitive(x) for x in n.xs))
    return n


# --------------------------------------------------------------------------
# combine model: a parser is f(s, pos) -> ("ok", value, newpos) | ("err", committed)
# --------------------------------------------------------------------------

OK, ERR = "ok", "err"
NON_ESCAPABLE = set(b"&;:,`~-_!@#%'\"")  # parser.rs:252-254


def _byte(x: int):
    def p(s, i):
        if i < len(s) and s[i] == x:
            return (OK, x, i + 1)
        return (ERR, False)
    return p


def _satisfy(pred):
    def p(s, i):
        if i < len(s) and pred(s[i]):
            return (OK, s[i], i + 1)
        return (ERR, False)
    return p


_letter = _satisfy(lambda b: (65 <= b <= 90) or (97 <= b <= 122))
_digit = _satisfy(lambda b: 48 <= b <= 57)
_any = _satisfy(lambda b: True)


def _seq(*ps):
    """Tuple parser: an error after any consumption is committed."""
    def p(s, i):
        vals = []
        j = i
        for q in ps:
            r = q(s, j)
            if r[0] == ERR:
                return (ERR, r[1] or j > i)
            vals.append(r[1])
            j = r[2]
        return (OK, tuple(vals), j)
    return p


def _choice(*ps):
    def p(s, i):
        for q in ps:
            r = q(s, i)
            if r[0] == OK:
                return r
            if r[1]:
                return r
        return (ERR, False)
    return p


def _attempt(q):
    def p(s, i):
        r = q(s, i)
        if r[0] == ERR:
            return (ERR, False)
        return r
    return p


def _map(q, f):
    def p(s, i):
        r = q(s, i)
        if r[0] == ERR:
            return r
        return (OK, f(r[1]), r[2])
    return p


def _many(q, min1=False):
    def p(s, i):
        vals = []
        j = i
        while True:
            r = q(s, j)
            if r[0] == ERR:
                if r[1]:
                    return (ERR, True)
                break
            vals.append(r[1])
            j = r[2]
        if min1 and not vals:
            return (ERR, False)
        return (OK, vals, j)
    return p


def _optional(q):
    def p(s, i):
        r = q(s, i)
        if r[0] == OK:
            return r
        if r[1]:
            return r
        return (OK, None, i)
    return p


def _between(o, c, q):
    return _map(_seq(o, q, c), lambda v: v[1])


def _lazy(fn):
    def p(s, i):
        return fn()(s, i)
    return p


def _parse_digits(ds) -> int:
    # parser.rs:349-351: str::parse::<usize>().unwrap()
    if not ds:
        raise ReferencePanic("parse_digits: empty digit string")
    v = int(bytes(ds).decode())
    if v >= 1 << 64:
        raise ReferencePanic("parse_digits: usize overflow")
    return v


def _regex():
    # parser.rs:208-222
    return _choice(
        _attempt(_map(_seq(_term(), _byte(ord("|")), _lazy(_regex)),
                      lambda v: Node("Either", a=v[0], b=v[2]))),
        _term(),
    )


def _term():
    # parser.rs:224-236
    return _map(_many(_lazy(_factor)),
                lambda xs: xs[0] if len(xs) == 1 else Node("Seq", xs=tuple(xs)))


def _factor():
    # parser.rs:238-250
    return _choice(
        _map(_attempt(_seq(_atom(), _byte(ord("?")))), lambda v: Node("Optional", a=v[0])),
        _attempt(_repeated()),
        _atom(),
    )


_EXT = False  # grammar extension active (set by parse(..., ext=True))


def _when_ext(q):
    def p(s, i):
        return q(s, i) if _EXT else (ERR, False)
    return p


def _bracket():
    ref = _between(_byte(ord("[")), _byte(ord("]")), _lazy(_range))
    ext = _between(_byte(ord("[")), _byte(ord("]")), _lazy(_ext_class))

    def p(s, i):
        if not _EXT:
            return ref(s, i)
        return _choice(_attempt(ref), ext)(s, i)
    return p


def _atom():
    # parser.rs:256-269 (+ the extension's bare digits and classes)
    return _choice(
        _map(_byte(ord(".")), lambda _: Node("Any")),
        _map(_attempt(_map(_seq(_byte(ord("\\")), _any), lambda v: v[1])), lambda c: Node("Char", c=c)),
        _map(_choice(_letter, _satisfy(lambda b: b in NON_ESCAPABLE)), lambda c: Node("Char", c=c)),
        _map(_when_ext(_digit), lambda c: Node("Char", c=c)),
        _bracket(),
        _between(_byte(ord("(")), _byte(ord(")")), _lazy(_regex)),
    )


def _ext_class():
    # extension: class := '^' class | item+ ; item := cc '-' cc | cc
    cc = _choice(
        _attempt(_map(_seq(_byte(ord("\\")), _any), lambda v: v[1])),
        _satisfy(lambda b: (65 <= b <= 90) or (97 <= b <= 122) or (48 <= b <= 57)
                 or (b in NON_ESCAPABLE and b != ord("-"))),
    )

    def rng(v):
        if v[2] < v[0]:
            raise ParseError("character class range out of order")
        return (v[0], v[2])
    item = _choice(_attempt(_map(_seq(cc, _byte(ord("-")), cc), rng)), _map(cc, lambda c: (c, c)))
    return _choice(
        _map(_seq(_byte(ord("^")), _lazy(_ext_class)), lambda v: Node("Not", a=v[1])),
        _map(_many(item, min1=True), lambda its: Node("Class", cs=tuple(x for it in its for x in it))),
    )


def _range():
    # parser.rs:279-294
    return _choice(
        _map(_seq(_byte(ord("^")), _lazy(_range)), lambda v: Node("Not", a=v[1])),
        _attempt(_map(_seq(_letter, _byte(ord("-")), _letter), lambda v: Node("Between", f=v[0], t=v[2]))),
        _map(_many(_letter, min1=True), lambda cs: Node("Range", cs=tuple(cs))),
    )


def _repeated():
    # parser.rs:296-347
    def rep_quant(v):
        re, c = v
        return Node("Repeated", a=re, lo=None if c == ord("*") else 1, hi=None)

    def rep_exact(v):
        re, ds = v
        n = _parse_digits(ds)
        return Node("Repeated", a=re, lo=n, hi=n)

    def rep_range(v):
        re, (lo_ds, _, hi_ds) = v
        lo = None if len(lo_ds) == 0 else _parse_digits(lo_ds)
        hi = None if len(hi_ds) == 0 else _parse_digits(hi_ds)
        return Node("Repeated", a=re, lo=lo, hi=hi)

    return _choice(
        _map(_attempt(_seq(_atom(), _choice(_byte(ord("*")), _byte(ord("+"))))), rep_quant),
        _map(_attempt(_seq(_atom(), _between(_byte(ord("{")), _byte(ord("}")), _many(_digit)))), rep_exact),
        _map(_seq(_atom(), _between(_byte(ord("{")), _byte(ord("}")),
                                    _seq(_many(_digit), _byte(ord(",")), _many(_digit)))), rep_range),
    )


def parse(pattern: str | bytes, ext: bool = False) -> Node:
    """parser.rs:146-185 (ext: the grammar extension, see the module docstring)."""
    global _EXT
    prev, _EXT = _EXT, bool(ext)
    try:
        return _parse(pattern)
    finally:
        _EXT = prev


def _parse(pattern: str | bytes) -> Node:
    s = pattern.encode() if isinstance(pattern, str) else bytes(pattern)

    def wrap(v):
        sof, re, eof = v
        if sof is None and eof is None:
            return re
        xs = []
        if sof is not None:
            xs.append(Node("SOF"))
        xs.append(re)
        if eof is not None:
            xs.append(Node("EOF"))
        return Node("Seq", xs=tuple(xs))

    top = _seq(
        _map(_between(_byte(ord("/")), _byte(ord("/")),
                      _seq(_optional(_byte(ord("^"))), _regex(), _optional(_byte(ord("$"))))), wrap),
        _optional(_byte(ord("i"))),
    )
    r = top(s, 0)
    if r[0] == ERR:
        raise ParseError("failed to parse regular expression")
    (re, ci), rest = r[1], r[2]
    if ci is not None:
        re = case_insensitive(re)
    if rest != len(s):
        raise ParseError("failed to parse regular expression, unexpected token")
    return re


# --------------------------------------------------------------------------
# Execution (execution.rs) over plaintext values, hash-consed keys
# --------------------------------------------------------------------------

CT_FALSE, CT_TRUE = 0, 1


class Execution:
    def __init__(self, content: bytes):
        self.content = content
        self.cache = {}
        self.ct_ops = 0
        self.cache_hits = 0
        self._intern = {}
        self._tuples = []

    def key(self, *t) -> int:
        k = self._intern.get(t)
        if k is None:
            k = len(self._tuples)
            self._intern[t] = k
            self._tuples.append(t)
        return k

    def const_of(self, k: int):
        t = self._tuples[k]
        return t[1] if t[0] == "C" else None

    # execution.rs:197-210
    def ct_constant(self, c: int):
        return (c, self.key("C", c))

    def ct_true(self):
        return self.ct_constant(CT_TRUE)

    def ct_false(self):
        return self.ct_constant(CT_FALSE)

    def ct_pos(self, at: int):
        return (self.content[at], self.key("P", at))

    def _with_cache(self, k, f):
        # execution.rs:212-222
        if k in self.cache:
            self.cache_hits += 1
            return (self.cache[k], k)
        self.ct_ops += 1
        v = f()
        self.cache[k] = v
        return (v, k)

    def ct_eq(self, a, b):  # :64-79 (smart_eq)
        return self._with_cache(self.key("=", a[1], b[1]), lambda: int(a[0] == b[0]))

    def ct_ge(self, a, b):  # :81-96 -- calls smart_gt (strict) at :93
        return self._with_cache(self.key(">", a[1], b[1]), lambda: int(a[0] > b[0]))

    def ct_le(self, a, b):  # :98-113
        return self._with_cache(self.key("<", a[1], b[1]), lambda: int(a[0] <= b[0]))

    def ct_and(self, a, b):  # :115-146
        k = self.key("&", a[1], b[1])
        ca, cb = self.const_of(a[1]), self.const_of(b[1])
        if ca == CT_TRUE:
            return (b[0], k)
        if ca == CT_FALSE:
            return (a[0], k)
        if cb == CT_TRUE:
            return (a[0], k)
        if cb == CT_FALSE:
            return (b[0], k)
        return self._with_cache(k, lambda: a[0] & b[0])

    def ct_or(self, a, b):  # :148-176
        k = self.key("|", a[1], b[1])
        ca, cb = self.const_of(a[1]), self.const_of(b[1])
        if ca == CT_TRUE:
            return (a[0], k)
        if cb == CT_TRUE:
            return (b[0], k)
        if ca == CT_FALSE and cb == CT_FALSE:
            return (a[0], k)
        return self._with_cache(k, lambda: a[0] | b[0])

    def ct_not(self, a):  # :178-195 (smart_bitxor with trivial 1)
        return self._with_cache(self.key("!", a[1]), lambda: a[0] ^ 1)


Lazy = Callable[[Execution], tuple]


def _seq_and(prev: Lazy, x: Lazy) -> Lazy:
    def f(ex):
        rp = prev(ex)
        rx = x(ex)
        return ex.ct_and(rp, rx)
    return f


def build_branches(L: int, re: Node, p: int) -> List[Tuple[Lazy, int]]:
    """engine.rs:45-214 (content only matters through its length here)."""
    k = re.kind
    if k == "SOF":
        return [(lambda ex: ex.ct_true(), p)] if p == 0 else []
    if k == "EOF":
        return [(lambda ex: ex.ct_true(), p)] if p == L else []
    if p >= L:
        return []
    if k == "Char":
        c = re.c
        return [(lambda ex, c=c, p=p: ex.ct_eq(ex.ct_pos(p), ex.ct_constant(c)), p + 1)]
    if k == "Any":
        return [(lambda ex: ex.ct_true(), p + 1)]
    if k == "Not":
        out = []
        for (br, e) in build_branches(L, re.a, p):
            out.append((lambda ex, br=br: ex.ct_not(br(ex)), e))
        return out
    if k == "Either":
        return build_branches(L, re.a, p) + build_branches(L, re.b, p)
    if k == "Between":
        f_, t_ = re.f, re.t

        def between(ex, p=p, f_=f_, t_=t_):
            ct_from = ex.ct_constant(f_)
            ct_to = ex.ct_constant(t_)
            ge = ex.ct_ge(ex.ct_pos(p), ct_from)
            le = ex.ct_le(ex.ct_pos(p), ct_to)
            return ex.ct_and(ge, le)
        return [(between, p + 1)]
    if k == "Range":
        cs = re.cs

        def rng(ex, p=p, cs=cs):
            res = ex.ct_eq(ex.ct_pos(p), ex.ct_constant(cs[0]))
            for c in cs[1:]:
                e = ex.ct_eq(ex.ct_pos(p), ex.ct_constant(c))
                res = ex.ct_or(res, e)
            return res
        return [(rng, p + 1)]
    if k == "Class":  # extension: OR over items of [lo <= c <= hi]
        cs = re.cs

        def cls(ex, p=p, cs=cs):
            res = None
            for i in range(0, len(cs), 2):
                lo, hi = cs[i], cs[i + 1]
                if lo == hi:
                    item = ex.ct_eq(ex.ct_pos(p), ex.ct_constant(lo))
                else:  # c >= lo as ct_ge(c, lo - 1): ct_ge is strict (execution.rs:93)
                    ge = ex.ct_true() if lo == 0 else ex.ct_ge(ex.ct_pos(p), ex.ct_constant(lo - 1))
                    le = ex.ct_true() if hi == 255 else ex.ct_le(ex.ct_pos(p), ex.ct_constant(hi))
                    item = ex.ct_and(ge, le)
                res = item if res is None else ex.ct_or(res, item)
            return res
        return [(cls, p + 1)]
    if k == "Repeated":
        at_least = 0 if re.lo is None else re.lo
        at_most = (L - p) if re.hi is None else re.hi
        if at_least > at_most:
            return []
        res = [[(lambda ex: ex.ct_true(), p)] if at_least == 0 else [],
               build_branches(L, Node("Seq", xs=tuple([re.a] * max(1, at_least))), p)]
        for _ in range(at_least + 1, at_most + 1):
            nxt = []
            for (bp, bpos) in res[-1]:
                for (bx, xpos) in build_branches(L, re.a, bpos):
                    nxt.append((_seq_and(bp, bx), xpos))
            res.append(nxt)
        return [b for lst in res for b in lst]
    if k == "Optional":
        return build_branches(L, re.a, p) + [(lambda ex: ex.ct_true(), p)]
    if k == "Seq":
        if not re.xs:
            raise ReferencePanic("Seq{[]}: index out of bounds (engine.rs:189-190)")
        conts = build_branches(L, re.xs[0], p)
        for x in re.xs[1:]:
            nxt = []
            for (bp, bpos) in conts:
                for (bx, xpos) in build_branches(L, x, bpos):
                    nxt.append((_seq_and(bp, bx), xpos))
            conts = nxt
        return conts
    raise ReferencePanic("unmatched regex variant")


@dataclass
class MatchResult:
    result: int
    ct_ops: int
    cache_hits: int
    n_branches: int


def has_match(content: bytes | str, pattern: str, start_lo: int = 0, start_hi: Optional[int] = None,
              ext: bool = False) -> MatchResult:
    """engine.rs:8-42.  ``start_lo/start_hi`` restrict the start offsets (the
    multi-GPU shard of §8(e)); the defaults reproduce the reference."""
    if isinstance(content, str):
        content = content.encode()
    re = parse(pattern, ext)
    L = len(content)
    hi = L if start_hi is None else start_hi
    branches = []
    for i in range(start_lo, hi):
        branches.extend(b for (b, _) in build_branches(L, re, i))
    ex = Execution(content)
    if len(branches) <= 1:
        res = branches[0](ex) if branches else ex.ct_false()
    else:
        res = branches[0](ex)
        for br in branches[1:]:
            r = br(ex)
            res = ex.ct_or(res, r)
    return MatchResult(res[0], ex.ct_ops, ex.cache_hits, len(branches))


# ---------------------------------------------------------------------------
# Position-set simulation (test oracle for the state-merging engine).  Same
# node rules as build_branches above, evaluated on plaintext: a map from
# content position to (OR of the branch values reaching it); presence of a key
# = some branch structurally reaches it.  Repetitions are run per visit
# position with the reference's exact count bounds (at_most = L - p when
# unbounded; lo = 0 allows at_most + 1).  Pinned against has_match on fuzzed
# patterns (tests/test_oracle.py).

def _char_ok(re: Node, ch: int) -> bool:
    k = re.kind
    if k == "Char":
        return ch == re.c
    if k == "Any":
        return True
    if k == "Between":  # ct_ge -> smart_gt (execution.rs:93)
        return ch > re.f and ch <= re.t
    if k == "Range":
        return ch in re.cs
    if k == "Class":
        return any(re.cs[i] <= ch <= re.cs[i + 1] for i in range(0, len(re.cs), 2))
    if k == "Not":
        return not _char_ok(re.a, ch)
    raise ValueError("Not over a multi-branch operand")


def _reach(L: int, content: bytes, re: Node, S: dict) -> dict:
    k = re.kind
    if k == "SOF":
        return {0: S[0]} if 0 in S else {}
    if k == "EOF":
        return {L: S[L]} if L in S else {}
    S = {p: v for p, v in S.items() if p < L}  # engine.rs:69-71
    if not S:
        return {}
    out: dict = {}

    def put(q, v):
        out[q] = out.get(q, False) or v

    if k in ("Char", "Any", "Between", "Range", "Class", "Not"):
        for p, v in S.items():
            put(p + 1, v and _char_ok(re, content[p]))
        return out
    if k == "Either":
        for d in (_reach(L, content, re.a, S), _reach(L, content, re.b, S)):
            for q, v in d.items():
                put(q, v)
        return out
    if k == "Optional":
        for q, v in _reach(L, content, re.a, S).items():
            put(q, v)
        for q, v in S.items():
            put(q, v)
        return out
    if k == "Seq":
        if not re.xs:
            raise ReferencePanic("Seq{[]}: index out of bounds (engine.rs:189-190)")
        cur = S
        for x in re.xs:
            cur = _reach(L, content, x, cur)
            if not cur:
                return {}
        return cur
    if k == "Repeated":
        for p, v in S.items():
            at_least = 0 if re.lo is None else re.lo
            at_most = (L - p) if re.hi is None else re.hi
            if at_least > at_most:
                continue
            if at_least == 0:
                put(p, v)
            first = max(1, at_least)
            last = first + (at_most - at_least)
            lev = {p: v}
            for kk in range(1, last + 1):
                lev = _reach(L, content, re.a, lev)
                if not lev:
                    break
                if kk >= first:
                    for q, w in lev.items():
                        put(q, w)
        return out
    raise ReferencePanic("unmatched regex variant")


def has_match_reach(content: bytes | str, pattern: str, start_lo: int = 0, start_hi: Optional[int] = None,
                    ext: bool = False) -> int:
    """Plaintext result of has_match by position-set simulation (polynomial)."""
    if isinstance(content, str):
        content = content.encode()
    re = parse(pattern, ext)
    L = len(content)
    hi = L if start_hi is None else min(start_hi, L)
    out = _reach(L, content, re, {p: True for p in range(start_lo, hi)})
    return int(any(out.values()))


if __name__ == "__main__":
    import json
    a = sys.argv[1:]
    r = has_match(a[0], a[1])
    print(json.dumps(r.__dict__))
