"""Which kernels ran inside bench.py's timed region, from a rocprofv3 kernel trace
of `BENCH_MARKERS=1 python bench.py ...` (two 1-cycle spin kernels mark t0 and the
end of the timed region; they are the first two spin kernels of the run).

usage: python tools/check_timed_window.py <dir with *kernel_trace.csv> [out.json]
"""
import collections
import csv
import glob
import json
import sys


def main(src, out=None):
    path = glob.glob(f'{src}/**/*kernel_trace.csv', recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    # the markers are 1-cycle spins (longer spins: the prep-stream probe, the
    # measurement window's launch cover)
    marks = [r for r in rows if ('spin' in r['Kernel_Name'] or 'sleep' in r['Kernel_Name'])
             and int(r['End_Timestamp']) - int(r['Start_Timestamp']) < 20000]
    if len(marks) < 2:
        raise SystemExit('no markers in trace (run bench.py with BENCH_MARKERS=1)')
    # the last two: the prep-stream probe's short spins come before the timed region
    t0, t1 = int(marks[-2]['Start_Timestamp']), int(marks[-1]['End_Timestamp'])
    inside = collections.Counter()
    before = collections.Counter()
    for r in rows:
        name = r['Kernel_Name'].split('(')[0]
        s = int(r['Start_Timestamp'])
        if t0 <= s <= t1:
            inside[name] += 1
        elif s < t0:
            before[name] += 1
    res = {'trace': path, 'timed_window_us': (t1 - t0) / 1e3,
           'kernels_inside': dict(inside.most_common()),
           'walk_launches_inside': sum(v for k, v in inside.items() if 'walk' in k),
           'sort_launches_inside': sum(v for k, v in inside.items() if 'sort' in k)}
    # launch timeline inside the window: offset from t0, duration, queue
    res['timeline'] = [
        '%9.1f %8.1f q%s %s' % ((int(r['Start_Timestamp']) - t0) / 1e3,
                               (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3,
                               r.get('Queue_Id', '?'), r['Kernel_Name'].split('(')[0][-60:])
        for r in rows if t0 <= int(r['Start_Timestamp']) <= t1]
    # with --hip-runtime-trace: the host API calls inside the window, interleaved
    # (offset, duration, 'H', name), and each kernel's launch-call offset
    api = glob.glob(f'{src}/**/*hip_api_trace.csv', recursive=True)
    if api:
        calls = sorted(csv.DictReader(open(api[0])), key=lambda r: int(r['Start_Timestamp']))
        launch_at = {r['Correlation_Id']: int(r['Start_Timestamp']) for r in calls}
        ev = [(int(r['Start_Timestamp']), '%9.1f %8.1f H  %s' % (
            (int(r['Start_Timestamp']) - t0) / 1e3,
            (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, r['Function']))
            for r in calls if t0 - 5000 <= int(r['Start_Timestamp']) <= t1]
        for r in rows:
            s = int(r['Start_Timestamp'])
            if t0 <= s <= t1:
                la = launch_at.get(r.get('Correlation_Id'))
                ev.append((s, '%9.1f %8.1f q%s %s (launched %+.1f)' % (
                    (s - t0) / 1e3, (int(r['End_Timestamp']) - s) / 1e3, r.get('Queue_Id', '?'),
                    r['Kernel_Name'].split('(')[0][-50:],
                    (la - t0) / 1e3 if la else float('nan'))))
        res['timeline'] = [e for _, e in sorted(ev)]
    print(json.dumps({k: v for k, v in res.items() if k != 'timeline'}, indent=1))
    print('\n'.join(res['timeline']))
    if out:
        json.dump(res, open(out, 'w'), indent=1)


if __name__ == '__main__':
    main(*sys.argv[1:])
