"""Summarise rocprofv3 SQ counter passes of bench.py (scripts/gpu_prof_r2.sh)
for the sampler kernel: counters per dispatch, per wave-step (one leapfrog
step of one wave's two chains in one slice) and as fractions of wave cycles.
    python scripts/pmc_sq.py <out.json> <kernel> <iters_per_launch> <L> [--floor F] <dir>...

Every averaged dispatch must be a launch of <iters_per_launch> iterations
(profile with --clock-warm-kind gemm --no-ess and warmup / steps multiples of
--iters-per-launch): a mix of launch sizes makes the per-wave-step figures
meaningless, so the script refuses dispatches whose SQ_INSTS_VALU (or
SQ_WAVE_CYCLES) differ by more than 20 %.  --floor F: the sweep's VALU per
wave-step (3 packed instructions per element of a lane's run), reported as
non_sweep_valu = VALU - F."""
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
    for c in ("SQ_INSTS_VALU", "SQ_WAVE_CYCLES"):
        v = out.get(c)
        if v and min(v) > 0 and max(v) / min(v) > 1.2:
            sys.exit(f"pmc_sq.py: {c} spans {min(v):.4g} .. {max(v):.4g} over {len(v)} dispatches "
                     f"of {match}: launches of different sizes are mixed")
    return ({c: sum(v) / len(v) for c, v in out.items()}, {c: len(v) for c, v in out.items()},
            {c: [min(v), max(v)] for c, v in out.items()})


def main():
    path, kern, ipl, L = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rest = sys.argv[5:]
    floor = None
    if rest and rest[0] == "--floor":
        floor, rest = float(rest[1]), rest[2:]
    avg, n, spread = collect(rest, kern)
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
           "dispatches_averaged": n, "dispatch_min_max": spread,
           "wave_steps_per_dispatch": ws,
           "counters_per_dispatch": avg, "per_wave_step": per_ws,
           "fractions_of_wave_cycles": frac,
           "note": "rocprofv3 --pmc, separate passes; cycle counters in the SQ's units"}
    if floor is not None and "SQ_INSTS_VALU" in per_ws:
        rec["sweep_floor_valu"] = floor
        rec["non_sweep_valu_per_wave_step"] = per_ws["SQ_INSTS_VALU"] - floor
    json.dump(rec, open(path, "w"), indent=1)
    print(json.dumps({"per_wave_step": per_ws, "fractions": frac}, indent=1))


if __name__ == "__main__":
    main()
