# Drop-in call-pattern lines (BASELINE configs 3-4 through the modules and hooks), Kaggle B=128.
# usage: bash tools/gpu_dropin.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
K="--config kaggle --batch-per-gpu 128 --steps 100 --warmup 10"
one() {  # <name> <args...>
  n=$1; shift
  timeout -k 10 300 python bench.py $K "$@" > gpurun_out/${T}_dropin_$n.log 2>&1 || { tail -n 30 gpurun_out/${T}_dropin_$n.log; exit 1; }
  tail -n 1 gpurun_out/${T}_dropin_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['us_per_step'], 'launches', d['launches_per_step'], 'direct', d['direct_api'], 'torch', d.get('torch_gpu_reference'))"
}
one sgd_list_sparse --mode dropin-sgd --dropin-form list --grad-mode sparse
one sgd_list_fused --mode dropin-sgd --dropin-form list --grad-mode fused_sgd
one sgd_coll_fused --mode dropin-sgd --dropin-form collection --grad-mode fused_sgd
one sgd_coll_sparse --mode dropin-sgd --dropin-form collection --grad-mode sparse
one dp_list --mode dropin-dp --dropin-form list
one dp_coll --mode dropin-dp --dropin-form collection
