"""Generates tests/golden/fuzz_scale.json: seeded random reference-grammar
patterns (tests/regex_fuzz.py) on random contents of 64-300 chars, with the
decrypted result the oracle's position-set simulator gives
(oracle/regex_oracle.py has_match_reach; polynomial, independent of the
enumerator and of the product's lowering).  The GPU test
(tests/test_gpu.py::test_fuzz_scale_vs_oracle) runs each case on encrypted
content: multi-launch levels, the throughput shape, deep circuits and plan
eviction on random circuits.  Patterns the reference rejects (Err / panic) are
skipped.  Run from the repo root: python3 tests/golden/make_fuzz_scale.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "..", "oracle")]
import regex_fuzz as rf  # noqa: E402
import regex_oracle as ro  # noqa: E402


def main(count=20, seed=2024):
    rng = random.Random(seed)
    cases = []
    while len(cases) < count:
        p = rf.rand_pattern(rng)
        n = rng.randint(64, 300)
        c = rf.rand_content(rng, n)
        try:
            exp = ro.has_match_reach(c, p)
        except (ro.ParseError, ro.ReferencePanic):
            continue
        cases.append({"pattern": p, "content": c, "expected": exp})
    with open(os.path.join(HERE, "fuzz_scale.json"), "w") as f:
        json.dump({"seed": seed, "generator": "tests/regex_fuzz.py rand_pattern / rand_content",
                   "oracle": "oracle/regex_oracle.py has_match_reach", "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
