"""C5 mismatch localisation: the C5 workload verified under each Miller lane mode / serial setting of the loaded
library (BLSGPU_LIB selects a variant); prints the mismatch count against the workload's expected results."""
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from lodestar_amd.native import Context  # noqa: E402

ctx = Context([0])
w, n, desc, _ = bench.build_workload(ctx, "C5", 0)
call = {k: v for k, v in w.items() if k != "expected" and not k.startswith("_")}
for lanes in (0, 1, 2):
    for serial in (0, 1):
        ctx.set_option("miller_lanes", lanes)
        ctx.set_option("serial", serial)
        got, st = ctx.verify_raw(**call, seed=bench.SEED)
        bad = np.nonzero(got != w["expected"])[0]
        print(f"lanes {lanes} serial {serial}: {len(bad)} mismatches {bad[:6]} retries {st.batch_retries}", flush=True)
ctx.close()
