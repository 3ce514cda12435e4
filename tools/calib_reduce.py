"""Reduce tools/calib_condense.sh passes: per output set, the condense
kernel's FETCH_SIZE / WRITE_SIZE per launch (KB -> bytes) against the exact
byte counts of tools/condense_probe.py.known_bytes."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def known(name):
    # same arithmetic as condense_probe.known_bytes (which needs torch + bench)
    nx, nu, N, batch = 4, 2, 30, 65536
    n = N * nu
    w = n * (n + 1) // 2
    if name != "H":
        w += n
    if name == "HfG":
        w += nx * nu * N * (N + 1) // 2
    if name == "HfGd":
        w += N * nx * n
    r = N * (nx * nx + nx * nu + nx) + nx + nx * nx * 2 + nu * nu
    return {"write": 4 * w * batch, "read": 4 * r * batch}


def counter(path, name):
    vals = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == name and "condense_kernel" in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]) * 1024)
    return sum(vals) / len(vals) if vals else None


out = {"method": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE, one pass each, condense_kernel<float,4> "
                 "at B=65536 (tools/condense_probe.py pmc SET); counter KB*1024 per launch vs the "
                 "exact bytes of the output set", "sets": {}}
root = sys.argv[1]
for s in ("H", "HfG", "HfGd"):
    k = known(s)
    f = counter(os.path.join(root, f"{s}_FETCH_SIZE"), "FETCH_SIZE")
    w = counter(os.path.join(root, f"{s}_WRITE_SIZE"), "WRITE_SIZE")
    out["sets"][s] = {"known_write": k["write"], "known_read": k["read"], "WRITE_SIZE": w,
                      "FETCH_SIZE": f,
                      "write_ratio": None if w is None else round(w / k["write"], 4),
                      "fetch_ratio": None if f is None else round(f / k["read"], 4)}
print(json.dumps(out, indent=1))
