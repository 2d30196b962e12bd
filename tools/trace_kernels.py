"""Per-launch durations of the kernel_timing (direct-launch) pass at the end of
a bench run under rocprofv3 --kernel-trace: the last `n` oac:: launches.
usage: python tools/trace_kernels.py <rocprof dir> [n] [skip-substrings,comma-separated]"""
import csv, glob, os, sys
d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 13
f = max(glob.glob(d + '/**/*_kernel_trace.csv', recursive=True), key=os.path.getmtime)
skip = sys.argv[3].split(',') if len(sys.argv) > 3 else []
r = [x for x in csv.DictReader(open(f)) if 'oac::' in x['Kernel_Name']
     and not any(k in x['Kernel_Name'] for k in skip)]
r.sort(key=lambda x: int(x['Start_Timestamp']))
tot = 0
for x in r[-n:]:
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    tot += (e - s) / 1e3
    nm = x['Kernel_Name'].split('(')[0].replace('void ', '')[:44]
    print(f"{nm:46s} dur {(e - s) / 1e3:8.2f} us  grid {x['Grid_Size_X']}")
print(f"sum {tot:.1f} us")
