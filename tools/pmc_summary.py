"""Summarise rocprofv3 --pmc CSV runs (one directory per counter pass) for one kernel."""
import collections
import csv
import glob
import sys

# usage: python tools/pmc_summary.py ROOT [KERNEL_PATTERN] - ROOT holds one directory per
# counter pass, each with the CSV output (run_counter_collection.csv) or the rocpd database
# (run_results.db) that rocprofv3 writes
root, pattern = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "lenet_fused_kernelILb1"
# --per-step N: the persistent launch runs many steps per dispatch - print each counter summed over
# every matching dispatch, divided by the N steps the run executed, instead of per-dispatch medians
per_step = int(sys.argv[sys.argv.index("--per-step") + 1]) if "--per-step" in sys.argv else 0
agg = collections.defaultdict(list)
for f in glob.glob(f"{root}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if pattern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(f"{root}/*/run_results.db"):
    import sqlite3

    db = sqlite3.connect(f)
    per = collections.defaultdict(float)  # (dispatch, counter) -> value summed over its instances
    for name, disp, cname, val in db.execute("select name, dispatch_id, counter_name, counter_value from pmc_events"):
        if pattern in name:
            per[(disp, cname)] += float(val)
    for (_, cname), v in per.items():
        agg[cname].append(v)
med = {k: (sum(v) / per_step if per_step else sorted(v)[len(v) // 2]) for k, v in agg.items()}
if per_step:
    print(f"(each counter summed over its {len(next(iter(agg.values()), []))} dispatches / {per_step} steps)")
for k in sorted(med):
    print(f"{k:28s} {'per step' if per_step else 'median'} {med[k]:12.4g}  (n={len(agg[k])})")
g = med.get
if g("SQ_WAVE_CYCLES"):
    wc = g("SQ_WAVE_CYCLES")
    print(f"\nwave-cycle split: waiting (s_waitcnt/barrier) {g('SQ_WAIT_ANY', 0) / wc:.0%}, "
          f"issue-stalled {g('SQ_WAIT_INST_ANY', 0) / wc:.0%}, issuing {g('SQ_ACTIVE_INST_ANY', 0) / wc:.0%}")
if g("SQ_LDS_IDX_ACTIVE"):
    print(f"LDS bank-conflict cycles / LDS active cycles: {g('SQ_LDS_BANK_CONFLICT', 0) / g('SQ_LDS_IDX_ACTIVE'):.0%}")
if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
    print(f"L2 hit rate: {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.0%}")
if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
    print(f"MFMA busy cycles (sum over SIMDs) / GPU active cycles: {g('SQ_VALU_MFMA_BUSY_CYCLES') / g('GRBM_GUI_ACTIVE'):.2f}")
