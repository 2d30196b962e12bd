"""Per-launch timeline of graph-replayed steps from a rocprofv3 kernel trace:
prints one 8-step graph replay (the middle of the timed region) with each
kernel's duration and the gap since the previous kernel ended.
usage: python tools/trace_graph.py <rocprof dir> [launches]"""
import csv, glob, os, sys
d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
f = max(glob.glob(d + '/**/*_kernel_trace.csv', recursive=True), key=os.path.getmtime)
r = [x for x in csv.DictReader(open(f)) if 'oac::' in x['Kernel_Name']]
r.sort(key=lambda x: int(x['Start_Timestamp']))
mid = len(r) // 2
seg = r[mid:mid + n]
t0 = int(seg[0]['Start_Timestamp'])
prev_end = None
for x in seg:
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    nm = x['Kernel_Name'].split('(')[0].replace('void ', '')[:40]
    print(f"{(s - t0) / 1e3:9.2f} {nm:42s} dur {(e - s) / 1e3:6.2f}  gap {gap:6.2f}  grid {x['Grid_Size_X']}")
    prev_end = e
print(f"span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us for {len(seg)} launches")
