"""K35 launches in a rocprofv3 kernel trace of bench.py (BENCH_MARKERS=1): inside the
timed window, per launch the duration and the gap from the previous kernel's end on
the K35 queue, quantiles; and what else ran during the K35 launches (other kernels
overlapping them in time: the prep stream).

usage: python tools/k35_gaps.py <trace dir>
"""
import csv
import glob
import sys

import numpy as np


def main(src):
    path = sorted(glob.glob(f'{src}/**/*kernel_trace.csv', recursive=True))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    marks = [r for r in rows if ('spin' in r['Kernel_Name'] or 'sleep' in r['Kernel_Name'])
             and int(r['End_Timestamp']) - int(r['Start_Timestamp']) < 20000]
    t0, t1 = int(marks[-2]['End_Timestamp']), int(marks[-1]['Start_Timestamp'])
    win = [r for r in rows if t0 <= int(r['Start_Timestamp']) and int(r['End_Timestamp']) <= t1]
    k35 = [r for r in win if 'bpr_adam_step_kernel' in r['Kernel_Name']]
    q = lambda x: np.round(np.quantile(np.asarray(x), [0.1, 0.5, 0.9, 1.0]), 2).tolist()
    dur = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in k35]
    qid = 'Queue_Id' if 'Queue_Id' in k35[0] else None
    same = [r for r in win if qid is None or r[qid] == k35[0][qid]]
    ends = {}
    prev_end = None
    gaps = []
    for r in same:
        if 'bpr_adam_step_kernel' in r['Kernel_Name'] and prev_end is not None:
            gaps.append((int(r['Start_Timestamp']) - prev_end) / 1e3)
        prev_end = int(r['End_Timestamp'])
    others = [r for r in win if r not in same]
    over = []
    for r in k35:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        over.append(sum(1 for o in others if int(o['Start_Timestamp']) < e and
                        int(o['End_Timestamp']) > s))
    names = {}
    for o in others:
        n = o['Kernel_Name'].split('(')[0][:60]
        names[n] = names.get(n, 0) + 1
    print('window_us', round((t1 - t0) / 1e3, 1), 'k35 launches', len(k35))
    print('k35 duration us q10/50/90/max', q(dur))
    print('gap before k35 (same queue) us', q(gaps) if gaps else None)
    print('other-queue kernels overlapping a k35: q', q(over))
    print('other-queue kernels in window:', sorted(names.items(), key=lambda x: -x[1])[:12])
    seq = [(r['Kernel_Name'].split('(')[0][:40], round((int(r['End_Timestamp']) -
            int(r['Start_Timestamp'])) / 1e3, 2)) for r in same[:40]]
    print('first kernels on the K35 queue:', seq)


if __name__ == '__main__':
    main(sys.argv[1])
