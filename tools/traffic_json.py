"""Reduce rocprofv3 FETCH_SIZE / WRITE_SIZE passes to HBM bytes per launch
per kernel role (bench.py --traffic keys).  FETCH_SIZE x 2 (gfx950, see
MI355X_MICROARCH.md "HBM"), KB -> bytes, averaged over dispatches."""
import collections
import csv
import json
import sys

# first match wins: the fp64 hand-off's kernels (empty launches when no
# instance is handed off) must not be averaged into the fp32 kernels' roles
ROLES = [("condense_kernel<double", "fallback64"), ("qp_wg_count_kernel", "fallback64"),
         ("condense_stream_kernel", "condense"), ("mpc_group_kernel", "mpc_box"), ("mpc_quad_kernel", "mpc_box"), ("mpc_box_kernel", "mpc_box"), ("box_quad_kernel", "solve_box"),
         ("box_gi_kernel", "solve_box"), ("condense_kernel", "condense"),
         ("condense_mfma_kernel", "condense"), ("condense_mfma_fh_kernel", "condense"), ("sweep_mfma_kernel", "sweep"), ("sweep_rows_kernel", "sweep"), ("qp_pf_kernel", "solve_pf"), ("qp_zf_kernel", "solve_zf"), ("ipm_", "ipm"),
         ("qp_wg_kernel", "solve_qp"),
         ("dual_range_kernel", "poly_solve"), ("bicycle_rti_kernel", "bicycle_rti")]


def role(name):
    for key, r in ROLES:
        if key in name:
            return r
    return None


def read(path, counter):
    acc = collections.defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") != counter:
                continue
            r = role(row.get("Kernel_Name", ""))
            if r:
                acc[r].append(float(row["Counter_Value"]))
    return {r: sum(v) / len(v) for r, v in acc.items()}


cfg, fpath, wpath = sys.argv[1], sys.argv[2], sys.argv[3]
f = read(fpath, "FETCH_SIZE")
w = read(wpath, "WRITE_SIZE")
out = {"config": int(cfg), "units": "bytes per launch", "method":
       "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes); 2*FETCH_SIZE + WRITE_SIZE, KB*1024"}
for r in sorted(set(f) | set(w)):
    fb, wb = 2 * f.get(r, 0.0) * 1024, w.get(r, 0.0) * 1024
    out[r] = round(fb + wb)
    out[r + "_read"] = round(fb)
    out[r + "_write"] = round(wb)
print(json.dumps(out))
