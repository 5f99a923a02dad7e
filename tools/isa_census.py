"""Instruction census of a device assembly file (hipcc --cuda-device-only -S): per function, total instructions,
v_mad_u64_u32, scratch, accvgpr moves and calls at each loop depth (LLVM's block comments).  Tooling only.
    python tools/isa_census.py file.s [function-substring ...]"""
import re
import sys
from collections import Counter, defaultdict


def census(path):
    fn, depth = None, 0
    cnt = defaultdict(lambda: defaultdict(Counter))
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            fn, depth = m.group(1), 0
            continue
        if fn is None:
            continue
        if re.match(r"^\.LBB\w+:", line) or line.startswith("; %bb"):
            m = re.search(r"Depth=(\d+)", line)
            depth = int(m.group(1)) if m else 0
        s = line.strip()
        if not s or s.startswith((".", ";")):
            continue
        cnt[fn][depth][s.split()[0]] += 1
    return cnt


if __name__ == "__main__":
    c = census(sys.argv[1])
    keys = sys.argv[2:]
    for f, byd in c.items():
        if keys and not any(k in f for k in keys):
            continue
        parts = []
        for d, cc in sorted(byd.items()):
            tot = sum(cc.values())
            mad = cc["v_mad_u64_u32"]
            scr = sum(v for k, v in cc.items() if k.startswith("scratch"))
            acc = sum(v for k, v in cc.items() if "accvgpr" in k)
            call = cc["s_swappc_b64"]
            parts.append(f"d{d}: {tot} (mad {mad}, scratch {scr}, acc {acc}, calls {call})")
        print(f[:60], " | ".join(parts))
