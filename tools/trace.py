"""Per-edge clocks of one step from a rocprofv3 kernel trace.

The drop-in step is one train() call's queued launches, so in the trace a
step is a burst of back-to-back kernels separated from the next by the host's
per-call work.  Bursts of exactly N kernels (the step's launch count) are the
steps; this prints the median-span one: each kernel's duration and the
gap from the previous kernel's end (the launch edge inside the graph), then
the burst's span and kernel sum, and the edge statistics over all bursts.

usage: python tools/trace.py <rocprof output dir> N [max gap inside a step, us]"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
cut = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
f = max(glob.glob(d + '/*/*_kernel_trace.csv'), key=os.path.getmtime)
r = [x for x in csv.DictReader(open(f)) if 'oac::' in x['Kernel_Name']]
r.sort(key=lambda x: int(x['Start_Timestamp']))
t0 = [int(x['Start_Timestamp']) for x in r]
t1 = [int(x['End_Timestamp']) for x in r]
bursts, cur = [], [0]
for i in range(1, len(r)):
    if (t0[i] - t1[i - 1]) / 1e3 > cut:
        bursts.append(cur)
        cur = []
    cur.append(i)
bursts.append(cur)
steps = [b for b in bursts if len(b) == n]
if not steps:
    sys.exit('no burst of %d kernels (gap cut %.1f us) in %s' % (n, cut, f))
span = lambda b: (t1[b[-1]] - t0[b[0]]) / 1e3
steps.sort(key=span)
b = steps[len(steps) // 2]
tot = 0.0
for j, i in enumerate(b):
    dur = (t1[i] - t0[i]) / 1e3
    gap = (t0[i] - t1[i - 1]) / 1e3 if j else 0.0
    tot += dur
    nm = r[i]['Kernel_Name'].split('(')[0].replace('void ', '')[:48]
    print(nm.ljust(50), 'dur %6.2f us  edge %5.2f us  wg %s grid %s'
          % (dur, gap, r[i]['Workgroup_Size_X'], r[i]['Grid_Size_X']))
print('median step of %d steps: span %.1f us, kernel sum %.1f us, %d edges %.2f us'
      % (len(steps), span(b), tot, n - 1, span(b) - tot))
edges = [(t0[i] - t1[i - 1]) / 1e3 for s in steps for i in s[1:]]
print('edges over all steps: median %.2f us, p10 %.2f, p90 %.2f'
      % (statistics.median(edges), sorted(edges)[len(edges) // 10],
         sorted(edges)[9 * len(edges) // 10]))
