"""Instruction mix of the loops of one kernel in a hipcc --save-temps .s file.

usage: python tools/asm_loop_stats.py file.s kernel_symbol_substring
For every loop header label inside the kernel, counts VALU / SALU / LDS /
VMEM / MFMA / waitcnt instructions between the header and its last back-edge.
"""
import collections
import re
import sys


def main(path, ksub):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and ksub in l and l.rstrip().endswith(":")
                 or (l.startswith("_Z") and ksub in l.split(":")[0]))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end + 1]
    heads = []
    for i, l in enumerate(body):
        if "Loop Header" not in l:
            continue
        j = i if l.startswith(".LBB") else i - 1  # the label may sit on the line above the comment
        if body[j].startswith(".LBB"):
            heads.append((j, body[j].split(":")[0]))
    for hi, lab in heads:
        back = [i for i, l in enumerate(body) if re.search(r"s_(c)?branch\w*\s+" + re.escape(lab) + r"\s*$", l)]
        back = [i for i in back if i > hi]
        if not back:
            continue
        c = collections.Counter()
        for l in body[hi:back[-1] + 1]:
            t = l.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            op = t[0]
            k = ("mfma" if op.startswith("v_mfma") else "valu" if op.startswith("v_") else
                 "wait" if op.startswith("s_waitcnt") else "salu" if op.startswith("s_") else
                 "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else op)
            c[k] += 1
        print(lab, "lines", back[-1] - hi, dict(c))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
