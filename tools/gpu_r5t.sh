# Round-5 (for the next round's plan): SQ wave / instruction-cache counters of the TB step-boundary
# kernel vs the update-only kernel, and a 2-rank gloo rehearsal of the N>1 bench path on one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5t}
A="--steps 20 --warmup 5 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
bash tools/pmc_sq.sh ${T}_next "$A" "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM" > gpurun_out/${T}_sq_next.txt 2>&1 || { tail -n 20 gpurun_out/${T}_sq_next.txt; exit 1; }
grep -i "coalesce" gpurun_out/${T}_sq_next.txt
bash tools/pmc_sq.sh ${T}_sep "$A --separate-forward" "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM" > gpurun_out/${T}_sq_sep.txt 2>&1 || { tail -n 20 gpurun_out/${T}_sq_sep.txt; exit 1; }
grep -i "coalesce\|emb_fwd" gpurun_out/${T}_sq_sep.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --dist-backend gloo $A > gpurun_out/${T}_gloo2.log 2>&1 || { tail -n 30 gpurun_out/${T}_gloo2.log; exit 1; }
grep "^{" gpurun_out/${T}_gloo2.log | tail -n 1 | cut -c1-600
