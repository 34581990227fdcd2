"""Per-kernel HBM bytes per launch from tools/prof_models_pmc.sh output
(FETCH_SIZE x2 + WRITE_SIZE, KB as reported; the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md §HBM/rocprofv3) -> profiles/<tag>_<cfg>_pmc.json."""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r['Kernel_Name']].append(float(r['Counter_Value']))
    return agg


def main(cfg, tag='r01', src='gpurun_out', dst='profiles'):
    base = os.path.join(src, f'pmc_{cfg}')
    fetch = per_kernel(glob.glob(os.path.join(base, 'FETCH_SIZE', '*counter_collection.csv'))[0])
    write = per_kernel(glob.glob(os.path.join(base, 'WRITE_SIZE', '*counter_collection.csv'))[0])
    out = {}
    for k in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0]))):
        f, w = fetch.get(k, []), write.get(k, [])
        fkb = sum(f) / len(f) if f else 0.0
        wkb = sum(w) / len(w) if w else 0.0
        out[k] = {'launches': max(len(f), len(w)), 'fetch_kb': round(fkb, 1),
                  'write_kb': round(wkb, 1),
                  'hbm_bytes_per_launch': round((2 * fkb + wkb) * 1024)}
    json.dump(out, open(os.path.join(dst, f'{tag}_{cfg}_pmc.json'), 'w'), indent=1)
    for k, v in list(out.items())[:8]:
        print(v['launches'], v['hbm_bytes_per_launch'], k[:100])


if __name__ == '__main__':
    main(*sys.argv[1:])
