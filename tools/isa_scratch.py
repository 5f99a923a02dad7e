"""Static scratch-access census of a device assembly file (hipcc --cuda-device-only -S): per function, scratch
loads/stores outside loops and at each loop depth (from LLVM's block comments), plus calls.  Tooling only.
    python tools/isa_scratch.py file.s"""
import re
import sys
from collections import defaultdict

fn = None
depth = 0
cnt = defaultdict(lambda: defaultdict(int))
for line in open(sys.argv[1]):
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
    if s.startswith("scratch_") or s.startswith("buffer_store") or s.startswith("buffer_load"):
        cnt[fn][f"d{depth}"] += 1
    elif s.startswith("s_swappc"):
        cnt[fn][f"call_d{depth}"] += 1
for f, c in cnt.items():
    print(f"{f[:60]:60s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
