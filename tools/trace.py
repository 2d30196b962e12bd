"""Summarise a rocprofv3 kernel trace: per-launch durations of one step."""
import csv, glob, sys
d = sys.argv[1]
import os; f = max(glob.glob(d + '/*/*_kernel_trace.csv'), key=os.path.getmtime)
r = list(csv.DictReader(open(f)))
r.sort(key=lambda x: int(x['Start_Timestamp']))
oac = [x for x in r if 'oac::' in x['Kernel_Name']]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
start = len(oac) - n * 30
tot = 0
for i in range(start, start + n):
    x = oac[i]
    dur = (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1000
    gap = (int(x['Start_Timestamp']) - int(oac[i - 1]['End_Timestamp'])) / 1000
    tot += dur
    nm = x['Kernel_Name'].split('(')[0].replace('void ', '')[:48]
    print(nm.ljust(50), 'dur %6.1f us  gap %5.1f  wg %s grid %s' % (dur, gap, x['Workgroup_Size_X'], x['Grid_Size_X']))
print('sum of kernel durations: %.1f us' % tot)
