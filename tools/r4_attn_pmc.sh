#!/bin/bash
# instruction mix of the short attention backward at the C2 shape (tools/attn_bench.py, one PMC pass of 8 SQ counters)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU -d gpurun_out/apmc -o run --output-format csv -- python3 tools/attn_bench.py --only c2 > gpurun_out/apmc.log 2>&1
echo rc=$?
python - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/apmc/run_counter_collection.csv")))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    w = d["SQ_WAVES"] or 1
    print(k, {c: round(v / n[(k, c)] / (w / n[(k, "SQ_WAVES")]), 1) for c, v in d.items() if c != "SQ_WAVES"}, "waves/disp", round(w / n[(k, "SQ_WAVES")]))
PY
