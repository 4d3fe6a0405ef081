"""Summarise rocprofv3 --pmc CSV passes into per-launch numbers for the engine's kernels.

Usage: python profiles/summarize_pmc.py <pmc_root> <out.json> [pixels_per_launch] [input]
<pmc_root> holds one sub-directory per pass (run_counter_collection.csv in each), as written by
profiles/pmc_passes.sh. HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are
in KB; on gfx950 FETCH_SIZE reports half of the bytes of a coalesced streaming read, so it is
doubled (our loads are 8 B/lane coalesced planes; the doubled figure matches the algorithmic
read bytes of the launch, which is the calibration).
"""
import collections
import csv
import glob
import json
import os
import sys


def main(root, out, px=None, input_mode='bands'):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for f in glob.glob(os.path.join(root, '*', 'run_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            name = ('analyze' if 'analyze' in k else 'resolve' if 'resolve' in k else
                    'index' if 'lt_index_kernel' in k else None)
            if name is None:
                continue
            per[name][r['Counter_Name']] += float(r['Counter_Value'])
            launches[(name, os.path.dirname(f))].add(r['Dispatch_Id'])
    res = {}
    for name, ctr in per.items():
        n = max(len(v) for (k, d), v in launches.items() if k == name)
        row = {c: v / n for c, v in ctr.items()}
        if 'FETCH_SIZE' in row:
            row['hbm_read_bytes'] = row['FETCH_SIZE'] * 1024 * 2
        if 'WRITE_SIZE' in row:
            row['hbm_write_bytes'] = row['WRITE_SIZE'] * 1024
        if 'hbm_read_bytes' in row and 'hbm_write_bytes' in row:
            row['hbm_bytes'] = row['hbm_read_bytes'] + row['hbm_write_bytes']
            if px:
                row['hbm_bytes_per_px'] = row['hbm_bytes'] / px
        row['launches'] = n
        res[name] = row
    res['_source'] = root
    # the kernel build the counters belong to (bench.py compares it with its own): the hash
    # pmc_passes.sh recorded when it collected them (its environment included: a phase-cut or A/B
    # run under LT_JIT_DEFINES etc. is another build), else computed now and marked so
    stamp = os.path.join(root, '_build.txt')
    if os.path.exists(stamp):
        res['_build'] = open(stamp).read().strip()
        res['_build_stamped'] = 'at collection (pmc_passes.sh)'
    else:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from land_trendr_amd._abi import build_hash
        res['_build'] = build_hash()
        res['_build_stamped'] = 'at summary time (no _build.txt)'

    res['_pixels_per_launch'] = px
    res['_input'] = input_mode
    json.dump(res, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None,
         sys.argv[4] if len(sys.argv) > 4 else 'bands')
