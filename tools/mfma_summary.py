"""Per-kernel MFMA utilisation from one rocprofv3 --pmc pass
(tools/mfma_counters.sh).  Averages each counter per dispatch of every
mpcqp kernel and derives:
  clk      = GRBM_GUI_ACTIVE / 8   (rocprofv3 sums the 8 XCDs) -- kernel cycles
  busy     = SQ_VALU_MFMA_BUSY_CYCLES / (clk * 1024) -- MFMA-busy fraction per SIMD
             (the counter sums the 4 SIMDs of each of the 256 CUs: normalised
             per CU it exceeds 1 on the sweep kernels)
  flops    = SQ_INSTS_VALU_MFMA_MOPS_F32 * 512        (one MOP = 512 flops)
  tflops   = flops / the average dispatch duration of the kernel trace (when given)
Usage: python tools/mfma_summary.py counter_collection.csv [kernel_trace.csv]"""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r.get("Kernel_Name", "")
    if "mpcqp" not in k:
        continue
    agg[k.split("(")[0][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = collections.defaultdict(list)
if len(sys.argv) > 2:
    for r in csv.DictReader(open(sys.argv[2])):
        k = r.get("Kernel_Name", "")
        if "mpcqp" in k:
            dur[k.split("(")[0][:70]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    clk = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    e = dict(dispatches=len(next(iter(d.values()))), counters={c: round(v, 1) for c, v in m.items()})
    if clk > 0:
        e["kernel_cycles"] = round(clk, 1)
        e["mfma_busy"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (clk * 1024), 4)
    e["mfma_f32_flops"] = m.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) * 512
    if dur.get(k):
        t = sum(dur[k]) / len(dur[k]) * 1e-9
        e["avg_duration_us"] = round(t * 1e6, 1)
        e["mfma_f32_tflops"] = round(e["mfma_f32_flops"] / t / 1e12, 2)
    out[k] = e
print(json.dumps(out, indent=1))
