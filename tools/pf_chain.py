"""Where the PF fill's level chain waits (kernel trace of bench.py --pf): for each level t, the gap
between the end of k_pf_level(t-1) and the start of k_pf_level(t), and whether the launch it waited
for was the span stream (k_pf_diag(t-1) ending inside the gap) or k_pf_iloop(t).
usage: python tools/pf_chain.py KERNEL_TRACE_CSV"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].replace("void ", "").split("(")[0]
    lev = [r for r in rows if name(r) == "k_pf_level"]
    diag = [r for r in rows if name(r) == "k_pf_diag"]
    il = [r for r in rows if name(r) == "k_pf_iloop"]
    # the first fill of the trace (bench.py --pf --steps 1 --warmup 0: the timed fill, then one
    # instrumented fill): its levels are the first n-2 k_pf_level launches, n-2 = launches / fills
    nlev = len(lev) // 2 if len(lev) % 2 == 0 else len(lev)
    lev = lev[:nlev]
    t0 = int(lev[0]["Start_Timestamp"])
    t1 = int(lev[-1]["End_Timestamp"])
    ends_d = sorted(int(r["End_Timestamp"]) for r in diag if t0 <= int(r["End_Timestamp"]) <= t1)
    ends_i = sorted(int(r["End_Timestamp"]) for r in il if t0 <= int(r["End_Timestamp"]) <= t1)
    gap_d = gap_i = gap_o = 0.0
    busy = 0.0
    for t in range(1, len(lev)):
        e0, s1 = int(lev[t - 1]["End_Timestamp"]), int(lev[t]["Start_Timestamp"])
        busy += int(lev[t]["End_Timestamp"]) - s1
        g = max(0, s1 - e0)
        # the last side launch ending inside the gap is what the level waited for
        d = max([x for x in ends_d if e0 <= x <= s1] or [0])
        i = max([x for x in ends_i if e0 <= x <= s1] or [0])
        if d and d >= i:
            gap_d += g
        elif i:
            gap_i += g
        else:
            gap_o += g
    span = int(lev[-1]["End_Timestamp"]) - t0
    print(f"levels {len(lev)}  chain span {span / 1e6:.2f} ms  level kernels busy {busy / 1e6:.2f} ms")
    print(f"gaps waiting on the span stream (k_pf_diag) {gap_d / 1e6:.2f} ms, on k_pf_iloop {gap_i / 1e6:.2f} ms, "
          f"other {gap_o / 1e6:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
