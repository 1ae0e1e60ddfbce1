"""INTEGRATION.md's Rust binding against include/fheregex.h.

A maintainer copies the binding into the reference crate (src/regex/gpu.rs), so a field or
parameter it misses is memory corruption there, not a typo: every `#[repr(C)]` struct must list
the C struct's fields in order, and every `fn fr_*` it declares must exist in the header with
the same parameter count.
"""
import os
import re

import fheregex as F

DOC = os.path.join(F.REPO, "INTEGRATION.md")


def _c_struct_fields(hdr, name):
    m = re.search(r"typedef struct \{((?:(?!typedef).)*?)\}\s*" + name + r";", hdr, re.S)
    assert m, name
    body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
    return [d.split()[-1] for d in body.split(";") if d.strip()]


def _rust_struct_fields(doc, name):
    m = re.search(r"pub struct " + name + r" \{(.*?)\n\}", doc, re.S)
    assert m, name
    body = re.sub(r"//[^\n]*", "", m.group(1))
    return re.findall(r"pub (\w+):", body)


def _c_params(hdr):
    out = {}
    flat = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    for m in re.finditer(r"\b(fr_\w+)\(([^;{]*?)\);", flat, re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_rust_structs_match_header():
    hdr = open(F.HEADER).read()
    doc = open(DOC).read()
    rust_names = {"poly_size": "N"}  # the Rust binding spells N out
    for c_name, r_name in (("fr_match_stats", "FrMatchStats"), ("fr_params", "FrParams")):
        c = _c_struct_fields(hdr, c_name)
        r = [rust_names.get(f, f) for f in _rust_struct_fields(doc, r_name)]
        assert r == c, (c_name, r, c)


def test_rust_functions_exist_with_their_arity():
    hdr = _c_params(open(F.HEADER).read())
    doc = open(DOC).read()
    found = 0
    for m in re.finditer(r"fn (fr_\w+)\(([^)]*)\)\s*->\s*c_int;", doc, re.S):
        name, args = m.group(1), m.group(2).strip()
        n = 0 if not args else args.count(",") + 1 - (1 if args.rstrip().endswith(",") else 0)
        assert name in hdr, name
        assert hdr[name] == n, (name, n, hdr[name])
        found += 1
    assert found >= 40
