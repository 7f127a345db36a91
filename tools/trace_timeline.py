"""Timeline of one training iteration (or any repeated launch sequence) from a rocprofv3
--kernel-trace CSV: per dispatch its start offset, duration and the idle gap before it on the
same queue, for the last iteration whose first kernel matches FIRST.
Usage: python tools/trace_timeline.py run_kernel_trace.csv [FIRST=t_prologue]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "t_prologue"
key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start_Timestamp_ns"
key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "End_Timestamp_ns"
ev = sorted(((int(r[key_s]), int(r[key_e]), r["Kernel_Name"], r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows))
starts = [i for i, e in enumerate(ev) if first in e[2]]
if len(starts) < 2:
    sys.exit(f"fewer than two '{first}' dispatches")
i0, i1 = starts[-2], starts[-1]
t0 = ev[i0][0]
last_end = {}
busy = 0
for s, e, n, q in ev[i0:i1]:
    gap = s - last_end.get(q, s)
    last_end[q] = max(last_end.get(q, 0), e)
    busy += e - s
    name = n.replace("void ", "").replace("(anonymous namespace)::", "")
    name = name[:name.index("(")] if "(" in name else name
    print(f"{(s - t0) / 1e3:9.1f} us  q{q:>3s}  dur {(e - s) / 1e3:8.1f}  gap {gap / 1e3:6.1f}  {name[:60]}")
span = max(e for _, e, _, _ in ev[i0:i1]) - t0
print(f"iteration span {span / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us")
