"""Per-step kernel breakdown of a timed window, from a rocprofv3 kernel trace of a
run whose timed region is bracketed by two 1-cycle spin kernels (bench.py with
BENCH_MARKERS=1, tools/bench_models.py with MODELS_MARKERS=1).

For every kernel launched inside the window: launches per step, mean duration, device
time per step; the kernels sorted by device time per step; the dominant one (largest
time per step); the sum of kernel time per step (<= the step's wall time: kernels of
one graph replay run back to back, gaps are launch boundaries).

usage: python tools/step_breakdown.py <trace dir> <steps in the window> [out.json]
"""
import collections
import csv
import glob
import json
import sys


def short(name):
    """Kernel name without the argument list (templates kept)."""
    depth = 0
    for i, ch in enumerate(name):
        if ch == '<':
            depth += 1
        elif ch == '>':
            depth -= 1
        elif ch == '(' and depth == 0:
            return name[:i].replace('void ', '')
    return name.replace('void ', '')


def breakdown(src, steps):
    path = sorted(glob.glob(f'{src}/**/*kernel_trace.csv', recursive=True))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    marks = [r for r in rows if ('spin' in r['Kernel_Name'] or 'sleep' in r['Kernel_Name'])
             and int(r['End_Timestamp']) - int(r['Start_Timestamp']) < 20000]
    if len(marks) < 2:
        raise SystemExit('no markers in the trace (MODELS_MARKERS=1 / BENCH_MARKERS=1)')
    t0, t1 = int(marks[-2]['End_Timestamp']), int(marks[-1]['Start_Timestamp'])
    dur = collections.defaultdict(list)
    for r in rows:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if t0 <= s and e <= t1:
            dur[short(r['Kernel_Name'])].append((e - s) / 1e3)
    table = []
    for name, d in dur.items():
        table.append({'kernel': name, 'launches_per_step': round(len(d) / steps, 3),
                      'avg_us': round(sum(d) / len(d), 2),
                      'us_per_step': round(sum(d) / steps, 2)})
    table.sort(key=lambda x: -x['us_per_step'])
    busy = sum(x['us_per_step'] for x in table)
    window = (t1 - t0) / 1e3
    return {'trace': path, 'steps': steps, 'window_us': round(window, 1),
            'wall_us_per_step': round(window / steps, 2),
            'kernel_us_per_step': round(busy, 2),
            'launches_per_step': round(sum(x['launches_per_step'] for x in table), 2),
            'dominant': table[0] if table else None, 'kernels': table}


if __name__ == '__main__':
    res = breakdown(sys.argv[1], int(sys.argv[2]))
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], 'w').write(txt)
    print(json.dumps({k: v for k, v in res.items() if k != 'kernels'}, indent=1))
    for x in res['kernels'][:25]:
        print('%8.2f us/step %6.2f x %8.2f us  %s' % (x['us_per_step'], x['launches_per_step'],
                                                       x['avg_us'], x['kernel'][:110]))
