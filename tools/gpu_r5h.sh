#!/bin/bash
# Round-5 session H: the N > 1 bench path rehearsed on one GPU (2 ranks sharing cuda:0 over gloo), default and MLS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5h
mkdir -p $O
export MIMI_BENCH_DIST_BACKEND=gloo
timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --cpu-baseline-seconds 0 --json-out $O/n2_b32.json > $O/n2_b32.log 2>&1 || { echo "n2 failed"; tail -20 $O/n2_b32.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/n2_b32.json')); print('n2', d['value'], d['n_gpus'], d['ms_per_step'], d['s8d_h2d_to_d2h']['value'], d['k32']['value'], d['b1_k8']['value'], d['per_utterance_k32']['value'])"
timeout -k 10 400 python -u bench.py --gpus 2 --workload mls --steps 3 --warmup 1 --cpu-baseline-seconds 0 --json-out $O/n2_mls.json > $O/n2_mls.log 2>&1 || { echo "n2 mls failed"; tail -20 $O/n2_mls.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/n2_mls.json')); print('n2 mls', d['value'], d['n_gpus'], d['ms_per_step'])"
