"""Gap analysis of a rocprofv3 csv trace: where the device idles inside one factorization."""
import csv, sys, re
from collections import defaultdict
d = sys.argv[1]; pre = sys.argv[2]
ks = list(csv.DictReader(open(f"{d}/{pre}_kernel_trace.csv")))
api = list(csv.DictReader(open(f"{d}/{pre}_hip_api_trace.csv")))
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[3] if len(sys.argv) > 3 else "k_q_anchors"
idx = [i for i, r in enumerate(ks) if anchor in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
# the window starts at the first kernel after the previous factorization's last kernel: take the api call gap
win = ks[a:b]
t0 = int(win[0]["Start_Timestamp"]); t1 = int(win[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
print(f"window {len(win)} kernels, span {(t1-t0)/1e6:.3f} ms, busy {busy/1e6:.3f} ms")
def short(n):
    n = re.sub(r"\(.*", "", n)
    if "rocprim" in n:
        m = re.findall(r"(radix_sort_onesweep_iteration|radix_sort_block_sort|onesweep_histogram|merge_sort_block_merge|block_sort|scan_impl|reduce|select|partition|init_lookback|scan_state)", n)
        n = "rocprim:" + (m[0] if m else "?")
    return n[-40:]
gaps = []
for p, q in zip(win, win[1:]):
    g = int(q["Start_Timestamp"]) - int(p["End_Timestamp"])
    gaps.append((g, short(p["Kernel_Name"]), short(q["Kernel_Name"]), int(p["End_Timestamp"]), int(q["Start_Timestamp"])))
print(f"sum gaps {sum(g for g,*_ in gaps)/1e6:.3f} ms")
apis = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in api]
agg = defaultdict(lambda: [0, 0])
for g, pn, qn, e, s in gaps:
    k = (pn, qn); agg[k][0] += g; agg[k][1] += 1
for k, (g, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:30]:
    # api calls inside such a gap
    print(f"{g/1e3:9.1f} us {c:4d}x  {k[0]:40s} -> {k[1]}")
# api time histogram inside window
at = defaultdict(lambda: [0, 0])
for s, e, f in apis:
    if s >= t0 and e <= t1: at[f][0] += e - s; at[f][1] += 1
print("host API inside window:")
for f, (t, c) in sorted(at.items(), key=lambda x: -x[1][0])[:15]:
    print(f"  {f:30s} {c:5d} calls {t/1e3:9.1f} us")
kt = defaultdict(lambda: [0, 0])
for r in win:
    kt[short(r["Kernel_Name"])][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"]); kt[short(r["Kernel_Name"])][1] += 1
print("kernels inside window:")
for f, (t, c) in sorted(kt.items(), key=lambda x: -x[1][0])[:25]:
    print(f"  {f:40s} {c:5d} calls {t/1e3:9.1f} us")
