"""Transcribe the reference README's documented regex semantics into a fixture.

Source: /root/reference/README.md:33-58 ("Supported regex constructs"): for each construct
the README names strings the pattern matches and (for "only matches") implies others it
does not.  Each entry: pattern, content, the README's claim (1 = match), and the README line.
The README's claims are the reference authors' statement of the engine's behaviour; the
code (src/regex/execution.rs:93: ct_ge calls smart_gt) deviates from two of them, recorded
in QUIRKS with the reason, so tests/test_oracle.py can pin the oracle to every other claim
and to the code's behaviour on those two.
Run: python tests/golden/make_readme_vectors.py  (writes tests/golden/readme_vectors.json)
"""
import json
import os

# (README line, pattern, strings it matches, strings the "only" rules out)
CLAIMS = [
    (34, "/abc/", ["abc", "123abc", "abc123", "123abc456"], ["ab", "acb", "xbc", ""]),
    (35, "/^abc/", ["abc", "abc123"], ["123abc", "xabc"]),
    (36, "/abc$/", ["abc", "123abc"], ["abc123", "abcx"]),
    (37, "/^abc$/", ["abc"], ["abcd", "xabc", "ab"]),
    (38, "/^abc$/i", ["abc", "Abc", "aBc", "abC", "ABc", "aBC", "AbC", "ABC"], ["abd", "ABCD"]),
    (39, "/^ab?c$/", ["abc", "ac"], ["abbc", "bc"]),
    (40, "/^ab*c$/", ["ac", "abc", "abbc", "abbbc"], ["ab", "bc", "abd"]),
    (41, "/^ab+c$/", ["abc", "abbc", "abbbc"], ["ac", "ab"]),
    (43, "/^ab{2}c$/", ["abbc"], ["abc", "abbbc"]),
    (44, "/^ab{3,}c$/", ["abbbc", "abbbbc", "abbbbbc"], ["abbc", "abc"]),
    (45, "/^ab{2,4}c$/", ["abbc", "abbbc", "abbbbc"], ["abc", "abbbbbc"]),
    (46, "/^ab|cd$/", ["ab", "cd"], ["abcd", "xab", "cdx"]),
    (47, "/^.$/", ["a", "b", "A", "B", "?"], ["", "ab"]),
    (49, "/^[abc]$/", ["a", "b", "c"], ["d", "ab"]),
    (50, "/^[a-d]$/", ["a", "b", "c", "d"], ["e", "z"]),
    (52, "/^[^abc]$/", ["d", "z", "?"], ["a", "b", "c"]),
    (53, "/^[^a-d]$/", ["e", "z"], ["a", "b", "c", "d"]),
    (55, "/^\\.$/", ["."], ["a", ""]),
    (56, "/^\\*$/", ["*"], ["a", "**"]),
]
# where the code differs from the README: Between's lower bound is strict because ct_ge
# calls smart_gt (src/regex/execution.rs:93), so [a-d] excludes 'a'
QUIRKS = {("/^[a-d]$/", "a"): 0, ("/^[^a-d]$/", "a"): 1}


def main():
    out = []
    for line, pat, pos, neg in CLAIMS:
        for c, claim in [(x, 1) for x in pos] + [(x, 0) for x in neg]:
            e = {"readme_line": line, "pattern": pat, "content": c, "readme": claim}
            if (pat, c) in QUIRKS:
                e["code"] = QUIRKS[(pat, c)]
                e["note"] = "ct_ge calls smart_gt (execution.rs:93): Between's lower bound is strict"
            out.append(e)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "readme_vectors.json")
    with open(path, "w") as f:
        json.dump({"source": "/root/reference/README.md:33-58", "cases": out}, f, indent=1)
    print(f"wrote {len(out)} cases to {path}")


if __name__ == "__main__":
    main()
