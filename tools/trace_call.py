"""Timeline of one call of a serial kernel trace (e.g. rocprofv3 --kernel-trace of tools/urgent_latency.py): kernels from the N-th-last k_hash_prep to
the next, with queue, start / end (us from the call's first kernel) and duration.
    python tools/trace_call.py gpurun_out/TAG/run_kernel_trace.csv [N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nth = int(sys.argv[2]) if len(sys.argv) > 2 else 3
names = [r["Kernel_Name"].split("(")[0] for r in rows]
idx = [i for i, n in enumerate(names) if n == "k_hash_prep"]
i0, i1 = idx[-nth], idx[-nth + 1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0 - 4:i1 - 2]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{r['Kernel_Name'].split('(')[0][:30]:30s} q{r['Queue_Id']:>3s} {s:9.1f} {e:9.1f} {e - s:8.1f}")
