"""Where does a bench step's idle GPU time sit?  

Reads the rocprofv3 CSVs of one run (`--kernel-trace --hip-trace
--output-format csv`), finds the largest gaps between consecutive kernels
on the device (end of one, start of the next, whatever stream), and prints
the HIP API calls that overlap each gap, longest first.

  python scripts/gap_trace.py <dir with *kernel_trace.csv and *hip_api_trace.csv> [top]
"""
import csv
import glob
import os
import sys


def rows(pattern):
    f = glob.glob(pattern, recursive=True)
    if not f:
        return []
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    ks = rows(os.path.join(d, "**", "*kernel_trace.csv"))
    api = rows(os.path.join(d, "**", "*hip_api_trace.csv"))
    if not ks:
        print("no kernel trace")
        return
    kt = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in ks)
    calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r.get("Thread_Id", ""))
                   for r in api)
    t0 = kt[0][0]
    span = (kt[-1][1] - t0) / 1e6
    busy_end = kt[0][1]
    gaps = []
    for s, e, name in kt[1:]:
        if s > busy_end:
            gaps.append((s - busy_end, busy_end, s, name))
        busy_end = max(busy_end, e)
    gaps.sort(reverse=True)
    idle = sum(g[0] for g in gaps) / 1e6
    print(f"kernels {len(kt)}  span {span:.1f} ms  idle {idle:.1f} ms in {len(gaps)} gaps")
    # kernels by name: launches, total and mean duration; how many run at once
    byk = {}
    for s, e, name in kt:
        v = byk.setdefault(name, [0, 0])
        v[0] += 1
        v[1] += e - s
    print(f"sum of kernel durations {sum(v[1] for v in byk.values()) / 1e6:.1f} ms (busy {span - idle:.1f} ms)")
    for name, (n, t) in sorted(byk.items(), key=lambda x: -x[1][1])[:20]:
        print(f"  {t / 1e6:10.2f} ms  {n:8d} x {t / n / 1e3:9.1f} us  {name}")
    for g, a, b, nxt in gaps[:top]:
        print(f"gap {g/1e6:8.2f} ms at +{(a-t0)/1e6:9.2f} ms, next kernel {nxt}")
        ov = [(min(e, b) - max(s, a), f, tid, e - s) for s, e, f, tid in calls if s < b and e > a]
        ov.sort(reverse=True)
        for o, f, tid, dur in ov[:6]:
            print(f"    {o/1e6:8.2f} ms of {f} (call {dur/1e6:.2f} ms, thread {tid})")
    tot = {}
    for s, e, f, tid in calls:
        tot[f] = tot.get(f, 0) + (e - s)
    print("HIP API time by function (ms):")
    for f, v in sorted(tot.items(), key=lambda x: -x[1])[:15]:
        print(f"  {v/1e6:10.2f}  {f}")


if __name__ == "__main__":
    main()
