"""HBM bytes of the gather_probe launches (tools/gather_probe.py) from two rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md §HBM: FETCH_SIZE counts the
128-B requests of a streaming read as 64 B -> x2, WRITE_SIZE exact; both in KB).
The probe's K3 launches come in two runs of equal length, C2 tables first, then the
2M-row tables; dispatch order tells them apart.

usage: python tools/gather_pmc.py <fetch dir> <write dir> <probe json> <out json>
"""
import csv
import glob
import json
import sys


def values(src):
    path = glob.glob(f'{src}/**/*counter_collection.csv', recursive=True)[0]
    rows = [r for r in csv.DictReader(open(path)) if 'bpr_fwd_bwd' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r.get('Dispatch_Id', r.get('Correlation_Id', 0))))
    return [float(r['Counter_Value']) for r in rows]


def main(fetch_dir, write_dir, probe_json, out):
    f, w = values(fetch_dir), values(write_dir)
    probe = json.load(open(probe_json))
    n = len(f) // len(probe)
    res = []
    for k, p in enumerate(probe):
        fk = f[k * n:(k + 1) * n]
        wk = w[k * n:(k + 1) * n]
        hbm = (2 * sum(fk) / len(fk) + sum(wk) / len(wk)) * 1024
        p = dict(p)
        p.update({'traffic': int(hbm), 'traffic_unit': 'HBM bytes per launch (PMC)',
                  'traffic_over_algorithmic': round(hbm / p['bytes_per_launch'], 3),
                  'hbm_gbs_measured': round(hbm / (p['launch_us'] * 1e-6) / 1e9, 1),
                  'fetch_kb': round(sum(fk) / len(fk), 1), 'write_kb': round(sum(wk) / len(wk), 1),
                  'launches_counted': len(fk)})
        res.append(p)
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:])
