"""Per-launch HBM traffic of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o pmc -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o pmc -- python bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_f gpurun_out/pmc_w 'gemm256_kernel<true, true>' 2433024 \
        profiles/r01_ff1_pmc.json

Units and corrections (MI355X_MICROARCH.md §HBM): both counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a 16-B/lane streaming read, so it is doubled; WRITE_SIZE is
exact for 16-B/lane stores.  FETCH_SIZE counts L2 misses including Infinity-Cache hits, so it
is an upper bound on HBM reads.  The dispatch is selected by kernel name and grid size (the
FF1 GEMM is the gemm256 NT instantiation with an 11 x 432 x 512-thread grid at B = 8).
"""
import csv
import json
import os
import sys


def values(d, kernel, grid):
    path = os.path.join(d, 'pmc_counter_collection.csv')
    out = []
    for r in csv.DictReader(open(path)):
        if kernel in r['Kernel_Name'] and r['Grid_Size'] == str(grid):
            out.append(float(r['Counter_Value']))
    return out


def main():
    fdir, wdir, kernel, grid, dst = sys.argv[1:6]
    f = values(fdir, kernel, grid)
    w = values(wdir, kernel, grid)
    assert f and w, 'no matching dispatches'
    fetch = 2.0 * 1024.0 * sum(f) / len(f)
    write = 1024.0 * sum(w) / len(w)
    res = {'kernel': kernel, 'grid_size': int(grid), 'dispatches': [len(f), len(w)],
           'fetch_bytes_per_launch': fetch, 'write_bytes_per_launch': write,
           'traffic_bytes_per_launch': fetch + write,
           'method': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; KiB x 1024; FETCH x2 (gfx950)'}
    json.dump(res, open(dst, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
