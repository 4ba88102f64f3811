set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/pmc.sh slp "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH" || exit 1
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob, collections
for p in sorted(glob.glob("gpurun_out/slp_p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(p)):
        if "k_hmc_sl" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(p)
    for k in acc: print(f"  {k:28s} {acc[k]/max(n[k],1):16.0f} per dispatch ({n[k]} dispatches)")
PY
