"""Per-kernel PMC table from rocprofv3 --pmc databases (one directory per counter pass).

usage: python tools/pmc_table.py ROOT [TOP]  - medians over each kernel's dispatches: waves,
wave-cycles per wave, VALU / MFMA / LDS / VMEM-read instructions per wave, the wave-cycle split
(waiting, issue-stalled, issuing) and LDS bank-conflict cycles / LDS active cycles."""
import collections
import glob
import sqlite3
import sys

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 16
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/*/run_results.db"):
    per = collections.defaultdict(float)
    for name, disp, cname, val in sqlite3.connect(f).execute(
            "select name, dispatch_id, counter_name, counter_value from pmc_events"):
        per[(name, disp, cname)] += val
    for (name, _, cname), v in per.items():
        vals[name][cname].append(v)


def short(n):
    n = n.replace("void ", "").replace("dnn::(anonymous namespace)::", "").replace("dnn::", "")
    return n.split("(")[0][:58]


rows = []
for name, d in vals.items():
    med = {k: sorted(v)[len(v) // 2] for k, v in d.items()}
    wc, w = med.get("SQ_WAVE_CYCLES", 0), med.get("SQ_WAVES", 1)
    if not wc:
        continue
    g = med.get
    rows.append((wc, short(name), w, wc / w, g("SQ_INSTS_VALU", 0) / w, g("SQ_INSTS_MFMA", 0) / w,
                 g("SQ_INSTS_LDS", 0) / w, g("SQ_INSTS_VMEM_RD", 0) / w, g("SQ_WAIT_ANY", 0) / wc,
                 g("SQ_WAIT_INST_ANY", 0) / wc, g("SQ_ACTIVE_INST_ANY", 0) / wc,
                 g("SQ_LDS_BANK_CONFLICT", 0) / max(1, g("SQ_LDS_IDX_ACTIVE", 1))))
rows.sort(reverse=True)
print(f"{'kernel (medians over dispatches)':58s} {'waves':>6s} {'cyc/w':>7s} {'valu/w':>7s} {'mfma/w':>6s} "
      f"{'lds/w':>6s} {'vmrd/w':>6s} {'wait':>5s} {'stall':>5s} {'issue':>5s} {'ldsc':>5s}")
for r in rows[:top]:
    print(f"{r[1]:58s} {r[2]:6.0f} {r[3]:7.0f} {r[4]:7.0f} {r[5]:6.0f} {r[6]:6.0f} {r[7]:6.0f} {r[8]:5.0%} "
          f"{r[9]:5.0%} {r[10]:5.0%} {r[11]:5.0%}")
