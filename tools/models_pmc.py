"""HBM bytes per launch of named kernels from two rocprofv3 PMC passes of the same
command (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md §HBM: FETCH_SIZE counts the
128-B requests of a streaming read as 64 B -> x2, WRITE_SIZE exact; both in KB).

usage: python tools/models_pmc.py <fetch dir> <write dir> <out json> <kernel substr>...
"""
import csv
import glob
import json
import sys


def per_kernel(src, names):
    path = glob.glob(f'{src}/**/*counter_collection.csv', recursive=True)[0]
    out = {n: [] for n in names}
    for r in csv.DictReader(open(path)):
        for n in names:
            if n in r['Kernel_Name']:
                out[n].append(float(r['Counter_Value']))
    return out


def main(fetch_dir, write_dir, out, *names):
    f, w = per_kernel(fetch_dir, names), per_kernel(write_dir, names)
    res = {}
    for n in names:
        if not f[n] or not w[n]:
            continue
        fk, wk = sum(f[n]) / len(f[n]), sum(w[n]) / len(w[n])
        res[n] = {'traffic': int((2 * fk + wk) * 1024), 'fetch_kb': round(fk, 1),
                  'write_kb': round(wk, 1), 'launches_counted': [len(f[n]), len(w[n])],
                  'unit': 'HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)'}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:])
