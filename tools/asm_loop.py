#!/usr/bin/env python3
"""Instruction mix of a kernel's main loop from hipcc's --save-temps assembly (gfx950 .s): the smallest backward-branch
region holding the given number of MFMAs.
    python3 tools/asm_loop.py <file.s> <kernel-symbol-substring> <mfma-per-loop> [--dump]"""
import collections
import re
import sys


def main():
    path, pat, nmfma = sys.argv[1], sys.argv[2], int(sys.argv[3])
    s = open(path).read()
    starts = [m.start() for m in re.finditer(r"^(_ZN\S*" + re.escape(pat) + r"\S*):", s, re.M)]
    for st in starts:
        name = s[st:s.find(":", st)]
        end = s.find("s_endpgm", st)
        body = s[st:end].splitlines()
        labels = {}
        for n, l in enumerate(body):
            m = re.match(r"(\.LBB\S+):", l.strip())
            if m:
                labels[m.group(1)] = n
        best = None
        for n, l in enumerate(body):
            m = re.match(r"\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
            if m and m.group(1) in labels and labels[m.group(1)] < n:
                loop = [x.strip() for x in body[labels[m.group(1)]:n + 1]
                        if x.strip() and not x.strip().startswith((";", "."))]
                if sum(1 for x in loop if x.startswith("v_mfma")) == nmfma and (best is None or len(loop) < len(best)):
                    best = loop
        if best is None:
            print(name, ": no loop with", nmfma, "MFMAs")
            continue
        c = collections.Counter(x.split()[0] for x in best)
        cat = lambda p: sum(v for k, v in c.items() if p(k))  # noqa: E731
        print(f"{name}\n  loop {len(best)}: mfma {nmfma}, valu {cat(lambda k: k.startswith('v_') and not k.startswith('v_mfma'))}, "
              f"salu {cat(lambda k: k.startswith('s_'))}, ds_read {cat(lambda k: k.startswith('ds_read'))}, "
              f"ds_write {cat(lambda k: k.startswith('ds_write'))}, vmem {cat(lambda k: k.startswith('buffer_'))}")
        print("  salu:", ", ".join(f"{k} {v}" for k, v in c.most_common() if k.startswith("s_")))
        if "--dump" in sys.argv:
            print("\n".join(best))


if __name__ == "__main__":
    main()
