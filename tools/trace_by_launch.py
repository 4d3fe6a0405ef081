"""Per-launch-shape summary of a rocprofv3 kernel trace (run_kernel_trace.csv): the analyze /
resolve kernels grouped by name and grid size, so the bench's 49 Mpx launches can be compared
with its HIP-event kernel time apart from the end-to-end and tiling legs' 16.8 Mpx launches.

    python tools/trace_by_launch.py <run_kernel_trace.csv> <bench.json> <out.json>
"""
import csv
import json
import sys


def main():
    trace, bench, out = sys.argv[1:4]
    groups = {}
    with open(trace) as fh:
        for r in csv.DictReader(fh):
            name = r['Kernel_Name']
            if not name.startswith('lt_'):
                continue
            ms = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
            groups.setdefault((name, int(r['Grid_Size_X'])), []).append(ms)
    b = json.load(open(bench))
    rows = [{'kernel': k, 'grid_x': g, 'launches': len(v), 'avg_ms': round(sum(v) / len(v), 3),
             'min_ms': round(min(v), 3), 'max_ms': round(max(v), 3)}
            for (k, g), v in sorted(groups.items())]
    res = {'command': 'rocprofv3 --kernel-trace --stats -- python3 bench.py (default: c2, timed '
                      'steps of one 49 Mpx launch + warmup, then the end-to-end and N>1-tiling '
                      'legs with 16.8 Mpx tiles)',
           'by_launch': rows,
           'bench_kernel_ms_hip_events': b['roofline'].get('kernel_ms')}
    with open(out, 'w') as fh:
        json.dump(res, fh, indent=1)
    for r in rows:
        print(r)


if __name__ == '__main__':
    main()
