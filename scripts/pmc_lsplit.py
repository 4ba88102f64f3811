"""Split a lane kernel's SQ instruction counts into the marginal leapfrog step
and the per-iteration remainder, from two instruction-mix passes that differ
only in L (scripts/gpu_round.sh sq1 TAG NAME --leapfrog L ...; every dispatch
of KERNEL in a pass is one launch of IPL iterations).

    python scripts/pmc_lsplit.py OUT.json KERNEL IPL WAVES L_A DIR_A L_B DIR_B [--floor F]

per_step[c] = (count_B - count_A) / ((L_B - L_A) * IPL * WAVES): what one more
leapfrog step costs a wave (the intermediate steps' mix); per_iteration[c] =
count_A / (IPL * WAVES) - L_A * per_step[c]: the momentum draws, the first /
last steps' extra items, the accept and the stores.  --floor: the sweep's
VALU per step (3 per element pair), reported as non_sweep_valu_per_step."""
import argparse
import collections
import csv
import glob
import json
import os


def counts(d, kernel):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        if kernel in r["Kernel_Name"]:
            per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for c, v in per.items():
        vals = sorted(v.values())
        if vals[-1] > 1.05 * vals[0]:  # (poll spins vary a little)
            raise SystemExit(f"{d}: {c} differs between dispatches {vals}: mixed launch sizes")
        out[c] = sum(vals) / len(vals)
    return out


ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("kernel")
ap.add_argument("ipl", type=int)
ap.add_argument("waves", type=int)
ap.add_argument("la", type=int)
ap.add_argument("da")
ap.add_argument("lb", type=int)
ap.add_argument("db")
ap.add_argument("--floor", type=float, default=0.0)
a = ap.parse_args()
A, B = counts(a.da, a.kernel), counts(a.db, a.kernel)
per_step, per_iter = {}, {}
for c in sorted(A):
    if c == "SQ_WAVES":
        continue
    ps = (B[c] - A[c]) / ((a.lb - a.la) * a.ipl * a.waves)
    per_step[c] = round(ps, 2)
    per_iter[c] = round(A[c] / (a.ipl * a.waves) - a.la * ps, 1)
rec = {"kernel": a.kernel, "iters_per_launch": a.ipl, "waves": a.waves,
       "passes": {str(a.la): a.da, str(a.lb): a.db},
       "per_step": per_step, "per_iteration": per_iter}
if a.floor:
    rec["sweep_floor_valu_per_step"] = a.floor
    rec["non_sweep_valu_per_step"] = round(per_step["SQ_INSTS_VALU"] - a.floor, 1)
for L in (a.la, a.lb, 20):
    rec[f"valu_per_wave_step_at_L{L}"] = round(per_step["SQ_INSTS_VALU"]
                                               + per_iter["SQ_INSTS_VALU"] / L, 1)
json.dump(rec, open(a.out, "w"), indent=1)
print(json.dumps(rec, indent=1))
