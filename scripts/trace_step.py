"""One step's kernel timeline from a rocprofv3 --kernel-trace (+ --runtime-trace)
run of bench.py: every kernel of the step that starts at the N-th
k_update_cphd_a launch (us from its start), its queue, and — with the HIP API
trace — when the host issued its launch call, so a gap shows whether the GPU
waited for the host or for a dependency.

usage: python scripts/trace_step.py <rocprofv3 output dir> [step index]
"""
import csv
import glob
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    kt = rows(f"{d}/**/*kernel_trace.csv")
    api = {r["Correlation_Id"]: r for r in rows(f"{d}/**/*hip_api_trace.csv")}
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(kt) if "update_cphd_a" in r["Kernel_Name"] or "update_phd_a" in r["Kernel_Name"]]
    if len(starts) < k + 2:
        sys.exit(f"only {len(starts)} steps traced")
    i0, i1 = starts[k], starts[k + 1]
    t0 = int(kt[i0]["Start_Timestamp"])
    # every kernel that starts in [part A(k), part A(k+1)] on any queue
    t_end = int(kt[i1]["Start_Timestamp"])
    print(f"step {k}: period {(t_end - t0) / 1e3:.1f} us; columns: start end dur (us from part A start), queue, "
          f"host launch call (us), kernel")
    for r in kt:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 or s > t_end:
            continue
        a = api.get(r["Correlation_Id"])
        host = f"{(int(a['Start_Timestamp']) - t0) / 1e3:9.1f}" if a else "        -"
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q {r.get('Queue_Id', '?'):>2}  {host}  "
              f"{r['Kernel_Name'].split('(')[0][:60]}")


def host_calls(d, k, lo_name="update_cphd_c", hi_name="k_predict"):
    """The HIP API calls the host made between the launch call of step k's part
    C and that of the next predict (what the context stream holds between them)."""
    kt = rows(f"{d}/**/*kernel_trace.csv")
    api = rows(f"{d}/**/*hip_api_trace.csv")
    by_corr = {r["Correlation_Id"]: r for r in api}
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(kt) if "update_cphd_a" in r["Kernel_Name"] or "update_phd_a" in r["Kernel_Name"]]
    t0 = int(kt[starts[k]]["Start_Timestamp"])
    c = next(r for r in kt[starts[k]:] if lo_name in r["Kernel_Name"])
    p = next(r for r in kt[starts[k]:] if hi_name in r["Kernel_Name"])
    a0 = int(by_corr[c["Correlation_Id"]]["Start_Timestamp"])
    a1 = int(by_corr[p["Correlation_Id"]]["Start_Timestamp"])
    print(f"host calls between the part C launch ({(a0 - t0) / 1e3:.1f}) and the next predict launch ({(a1 - t0) / 1e3:.1f}):")
    for r in sorted(api, key=lambda r: int(r["Start_Timestamp"])):
        s = int(r["Start_Timestamp"])
        if a0 <= s <= a1 and not r["Function"].startswith(("hipGetLastError", "hipSetDevice", "hipGetDevice")):
            print(f"  {(s - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - s) / 1e3:7.1f}  {r['Function']}")


if __name__ == "__main__":
    main()
    if len(sys.argv) > 3:
        host_calls(sys.argv[1], int(sys.argv[2]))
