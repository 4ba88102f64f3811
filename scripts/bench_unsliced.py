"""Unsliced programs: chain-per-workgroup kernel (k_hmc) against the one-slice
lane-resident kernel (k_hmc_lr, slice_kernel="lanes") over model size and
chain count.  Prints one JSON object {model: {chains: {kernel: M steps/s}}};
the timing is the sampling phase's device time (RunInfo.sampling_seconds)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as ge

    m = ge._ensure_pkg()
    import workloads as W

    ns = W.ns_product()
    models = {
        "simple_normal_n100": W.simple_normal(ns, 100),
        "iso_d10": W.iso_normal(ns, 10),
        "iso_d100": W.iso_normal(ns, 100),
        "hier_small_1k": W.hierarchical(ns, *W.SHAPES["small"]),
    }
    out = {}
    for name, (lp, init) in models.items():
        out[name] = {}
        for C in (64, 256, 1024):
            row = {}
            for kernel, slices in (("k_hmc", 1), ("lanes", 1)):
                L, ns_, nw = 10, 300, 100
                s, rate, info = m.hmc(lp, init, num_samples=ns_, num_warmup=nw, step_size=0.05,
                                      num_leapfrog_steps=L, key=m.random.key(0), num_chains=C,
                                      progress=False, return_info=True, num_slices=slices,
                                      slice_kernel="lanes" if kernel == "lanes" else "auto")
                row[kernel] = round(C * ns_ * L / info.sampling_seconds / 1e6, 2)
            out[name][C] = row
            print(name, C, row, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
