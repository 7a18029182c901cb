"""Per-level timeline of the prepass scheme (CCJ_PREPASS=1) from a rocprofv3 kernel trace: for each
level t, the plain launch (k_level4d) and the prepass leader launch of level t (the k_level4d_lead
dispatched after k_diag2d(t-1)), and what the plain launch waited for.
usage: python tools/prepass_timeline.py TRACE.csv [fold index, default -2]"""
import csv
import re
import statistics as stx
import sys


def kname(full):
    return re.sub(r"^void ", "", full.split("(")[0]).strip()


rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Dispatch_Id"]), kname(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows.sort()
which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
starts = [i for i, x in enumerate(rows) if x[1] == "k_init2d"] + [len(rows)]
fold = rows[starts[which - 1]:starts[which]] if which < 0 else rows[starts[which]:starts[which + 1]]
plain, pre, diag = [], {}, []
for x, (d, k, s, e) in enumerate(fold):
    if k == "k_diag2d":
        diag.append((s, e))
    elif k == "k_level4d":
        plain.append((s, e))
    elif k == "k_level4d_lead":
        pre[len(diag)] = (s, e)  # enqueued after k_diag2d(len(diag)-1): level len(diag)
t0 = fold[0][2]
gaps, waits = [], []
print("   t  plain_start  plain_us  pre_start  pre_us  pre_end-prev_plain_end")
for t in range(1, len(plain)):
    ps, pe = plain[t]
    prev_end = plain[t - 1][1]
    gaps.append(ps - prev_end)
    w = (pre[t][1] - prev_end) if t in pre else None
    if w is not None:
        waits.append(w)
    if t % 10 == 0:
        print("%4d %10.1f %8.1f %10s %7s %8s" % (t, (ps - t0) / 1e3, (pe - ps) / 1e3,
              "%.1f" % ((pre[t][0] - t0) / 1e3) if t in pre else "-", "%.1f" % ((pre[t][1] - pre[t][0]) / 1e3) if t in pre else "-",
              "%.1f" % (w / 1e3) if w is not None else "-"))
print("fold %.2f ms; plain spans %.2f ms; gaps between plain launches %.2f ms; pre late (after prev plain end) on %d levels, sum %.2f ms"
      % ((max(r[3] for r in fold) - t0) / 1e6, sum(e - s for s, e in plain) / 1e6, sum(gaps) / 1e6,
         sum(1 for w in waits if w > 0), sum(w for w in waits if w > 0) / 1e6))
