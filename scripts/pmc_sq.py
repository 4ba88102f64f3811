"""Summarise rocprofv3 SQ counter passes of bench.py (scripts/gpu_prof_r2.sh)
for the sampler kernel: counters per dispatch, per wave-step (one leapfrog
step of one wave's two chains in one slice) and as fractions of wave cycles.
    python scripts/pmc_sq.py <out.json> <kernel> <iters_per_launch> <L> <dir>..."""
import csv
import glob
import json
import os
import sys


def collect(dirs, match):
    per = {}
    for d in dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                if match not in r["Kernel_Name"]:
                    continue
                key = (d, r["Dispatch_Id"])
                per.setdefault(key, {})
                c = r["Counter_Name"]
                per[key][c] = per[key].get(c, 0.0) + float(r["Counter_Value"])
    out = {}
    for (d, _), cs in per.items():
        for c, v in cs.items():
            out.setdefault(c, []).append(v)
    return {c: sum(v) / len(v) for c, v in out.items()}, {c: len(v) for c, v in out.items()}


def main():
    path, kern, ipl, L = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    avg, n = collect(sys.argv[5:], kern)
    waves = avg.get("SQ_WAVES", 0.0)
    ws = waves * ipl * L
    per_ws = {c: avg[c] / ws for c in avg if c.startswith("SQ_INSTS")} if ws else {}
    cyc = avg.get("SQ_WAVE_CYCLES")
    frac = {}
    if cyc:
        frac = {"valu_active": avg.get("SQ_ACTIVE_INST_VALU", 0) / cyc,
                "any_active": avg.get("SQ_ACTIVE_INST_ANY", 0) / cyc,
                "waiting": avg.get("SQ_WAIT_ANY", 0) / cyc}
    rec = {"kernel": kern, "iters_per_launch": ipl, "leapfrog_steps": L,
           "dispatches_averaged": n, "wave_steps_per_dispatch": ws,
           "counters_per_dispatch": avg, "per_wave_step": per_ws,
           "fractions_of_wave_cycles": frac,
           "note": "rocprofv3 --pmc, separate passes; cycle counters in the SQ's units"}
    json.dump(rec, open(path, "w"), indent=1)
    print(json.dumps({"per_wave_step": per_ws, "fractions": frac}, indent=1))


if __name__ == "__main__":
    main()
