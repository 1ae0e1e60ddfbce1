"""Instruction mix of a kernel's loops from the hipcc -save-temps ISA
(fhe-regex_amd: make asm).  Usage: python tools/isa_loop.py <func-substring> [file.s]"""
import collections
import re
import sys

def main():
    pat = sys.argv[1]
    path = sys.argv[2] if len(sys.argv) > 2 else "fhe-regex_amd/build/asm/device-hip-amdgcn-amd-amdhsa-gfx950.s"
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + pat + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:c)?branch\w*\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    for a, b in sorted(loops, key=lambda x: x[0] - x[1])[:3]:
        cnt = collections.Counter()
        for l in body[a:b + 1]:
            t = l.strip()
            if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
                continue
            cnt[t.split()[0]] += 1
        total = sum(cnt.values())
        print(f"loop lines {a}-{b}: {total} instructions")
        for k, v in cnt.most_common(40):
            print(f"  {v:6d} {k}")

main()
