"""Summarise a tools/prof_pmc.sh run (gpurun_out/prof/) into profiles/.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.json           per kernel: launches, mean FETCH_SIZE / WRITE_SIZE
                                    (KB as reported) and HBM bytes per launch with the
                                    gfx950 correction (MI355X_MICROARCH.md §HBM/rocprofv3:
                                    FETCH_SIZE counts 128-B requests as 64 B -> x2;
                                    WRITE_SIZE exact)
  profiles/<tag>_bench.json         the bench line of the traced run
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r['Kernel_Name']].append(float(r['Counter_Value']))
    return agg


def main(tag='r01', src='gpurun_out/prof', dst='profiles'):
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, 'trace', '*kernel_stats.csv'))[0]
    shutil.copy(stats, os.path.join(dst, f'{tag}_kernel_stats.csv'))
    fetch = per_kernel(glob.glob(os.path.join(src, 'fetch', '*counter_collection.csv'))[0])
    write = per_kernel(glob.glob(os.path.join(src, 'write', '*counter_collection.csv'))[0])
    out = {}
    for k in sorted(set(fetch) | set(write), key=lambda k: -sum(write.get(k, [0]))):
        f, w = fetch.get(k, []), write.get(k, [])
        fkb = sum(f) / len(f) if f else 0.0
        wkb = sum(w) / len(w) if w else 0.0
        out[k] = {'launches': max(len(f), len(w)), 'fetch_kb': round(fkb, 1),
                  'write_kb': round(wkb, 1),
                  'hbm_bytes_per_launch': round((2 * fkb + wkb) * 1024)}
    valu = glob.glob(os.path.join(src, 'valu', '*counter_collection.csv'))
    if valu:                                    # per-launch means of each SQ counter
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(valu[0])):
            agg[r['Kernel_Name']][r['Counter_Name']] += float(r['Counter_Value'])
            if 'Start_Timestamp' in r:
                disp[r['Kernel_Name']][r['Dispatch_Id']] = (
                    int(r['End_Timestamp']) - int(r['Start_Timestamp']))
        for k, cs in agg.items():
            n = max(len(disp[k]), 1)
            rec = {'valu_launches': n, **{c.lower() + '_per_launch': round(v / n, 1)
                                          for c, v in cs.items()}}
            # VALU pipe occupancy: SQ_ACTIVE_INST_VALU counts quad-cycles summed over
            # the waves; one SIMD issues one VALU instruction at a time, so
            # 4 * ACTIVE_INST_VALU / (SIMDs * clock * duration) is the fraction of the
            # chip's VALU issue time the kernel kept busy (1,024 SIMDs, 2.4 GHz)
            dur = sum(disp[k].values())
            if dur and 'SQ_ACTIVE_INST_VALU' in cs:
                rec['valu_busy_frac'] = round(4 * cs['SQ_ACTIVE_INST_VALU'] /
                                              (1024 * 2.4 * dur), 4)
                rec['pmc_duration_ns_per_launch'] = round(dur / n, 1)
            out.setdefault(k, {}).update(rec)
    json.dump(out, open(os.path.join(dst, f'{tag}_pmc.json'), 'w'), indent=1)
    for line in open(os.path.join(src, 'trace.log')):
        if line.startswith('{"metric"'):
            json.dump(json.loads(line), open(os.path.join(dst, f'{tag}_bench.json'), 'w'),
                      indent=1)
    print('wrote', dst, tag)


if __name__ == '__main__':
    main(*sys.argv[1:])
