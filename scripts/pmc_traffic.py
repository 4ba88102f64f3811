"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into
profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

HBM bytes per launch of the dominant kernel = (2 * FETCH_SIZE + WRITE_SIZE) * 1024:
FETCH_SIZE and WRITE_SIZE are kilobytes; on gfx950 FETCH_SIZE counts half the
bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section), so it is
doubled.  Usage:
    python scripts/pmc_traffic.py <fetch_dir> <write_dir> <key> <iters per launch> [label]
        [--kernel NAME] [--out PATH]
Records are keyed "<key>@<iters per launch>" (bench.py pmc_traffic; key =
the HMC shape, or "nuts-<model>-<shape>" / "mh-<shape>"): a launch's fixed
bytes (the slice blocks, once per launch) do not scale.  --out: the JSON file
to merge the record into (default profiles/pmc_traffic.json)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter, match):
    vals = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if match in r["Kernel_Name"] and r["Counter_Name"] == counter:
                key = r["Dispatch_Id"]
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return vals


KERNELS = ("k_hmc_lf", "k_hmc_lr", "k_hmc_sl", "k_nuts_lr", "k_nuts_sl", "k_mh_sl", "k_hmc",
           "k_nuts", "k_mh")


def main():
    args = list(sys.argv[1:])
    opts = {}
    for o in ("--kernel", "--out"):
        if o in args:
            i = args.index(o)
            opts[o] = args[i + 1]
            del args[i:i + 2]
    fdir, wdir, shape = args[0], args[1], args[2]
    ipl = int(args[3]) if len(args) > 3 else 1  # bench.py --iters-per-launch
    f = {}
    for kern in ([opts["--kernel"]] if "--kernel" in opts else KERNELS):  # the sampler kernel
        f = per_dispatch(fdir, "FETCH_SIZE", kern)
        if f:
            break
    if not f:
        sys.exit(f"pmc_traffic.py: no FETCH_SIZE record of {opts.get('--kernel', KERNELS)}")
    w = per_dispatch(wdir, "WRITE_SIZE", kern)
    fk = sum(f.values()) / max(len(f), 1)
    wk = sum(w.values()) / max(len(w), 1)
    out_path = opts.get("--out", os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    key = f"{shape}@{ipl}"
    data.pop(shape, None)  # (round-2 records were keyed by shape alone)
    data[key] = {
        "kernel": kern,
        "dispatches": [len(f), len(w)],
        "fetch_kb_min_max": [min(f.values()), max(f.values())],
        "iters_per_launch": ipl,
        "fetch_kb_per_launch": fk,
        "write_kb_per_launch": wk,
        "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0,
        "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)",
        "profile": args[4] if len(args) > 4 else "",
    }
    json.dump(data, open(out_path, "w"), indent=1)
    print(json.dumps(data[key]))


if __name__ == "__main__":
    main()
