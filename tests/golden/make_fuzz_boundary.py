"""Generates tests/golden/fuzz_boundary.json: seeded random reference-grammar
patterns (tests/regex_fuzz.py) on random contents of 256-512 chars in which a
short string the pattern matches -- or a one-character mutation of it, a near
miss -- is planted at the first or the last start offsets (engine.rs:15-18
enumerates every start; anchors, engine.rs:51-57, pin the ends), with the
decrypted result the oracle's position-set simulator gives
(oracle/regex_oracle.py has_match_reach; polynomial, independent of the
enumerator and of the product's lowering).  The GPU test
(tests/test_gpu.py::test_fuzz_boundary_vs_oracle) runs each case on encrypted
content.  Patterns the reference rejects (Err / panic) are skipped.
Run from the repo root: python3 tests/golden/make_fuzz_boundary.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "..", "oracle")]
import regex_fuzz as rf  # noqa: E402
import regex_oracle as ro  # noqa: E402

ALPHA = "abcdeABCxyz0.* "


def witness(rng, p, tries=400):
    """A short string on which p matches, found by sampling (None if none found)."""
    for _ in range(tries):
        s = "".join(rng.choice(ALPHA) for _ in range(rng.randint(1, 6)))
        if ro.has_match_reach(s, p):
            return s
    return None


def main(count=30, seed=4242):
    rng = random.Random(seed)
    cases = []
    while len(cases) < count:
        p = rf.rand_pattern(rng)
        try:
            ro.has_match_reach("a", p)
        except (ro.ParseError, ro.ReferencePanic):
            continue
        w = witness(rng, p)
        if w is None:
            continue
        n = rng.randint(256, 512)
        c = list(rf.rand_content(rng, n))
        plant = w
        if rng.random() < 0.4:  # near miss: one character of the witness changed
            i = rng.randrange(len(w))
            plant = w[:i] + rng.choice([ch for ch in ALPHA if ch != w[i]]) + w[i + 1:]
        at = 0 if rng.random() < 0.5 else n - len(plant)
        c[at:at + len(plant)] = plant
        c = "".join(c)
        cases.append({"pattern": p, "content": c, "planted": plant, "at": at, "expected": ro.has_match_reach(c, p)})
    with open(os.path.join(HERE, "fuzz_boundary.json"), "w") as f:
        json.dump({"seed": seed, "generator": "tests/regex_fuzz.py rand_pattern / rand_content + planted witness",
                   "oracle": "oracle/regex_oracle.py has_match_reach", "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
