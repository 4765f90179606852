# rocprofv3 evidence of one round in one GPU call: kernel trace + FETCH_SIZE / WRITE_SIZE
# passes (tools/prof_cfg.sh) of the TB and Kaggle N=1 lines and of the config-3 (B=128 SGD)
# line, summarised by tools/prof_summary.py into gpurun_out/<tag>_{tb,kaggle,c3}_*.
# usage: bash tools/gpu_profiles.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1
cd $R && mkdir -p gpurun_out
bash tools/prof_cfg.sh ${T}_tb terabyte || { tail -n 20 gpurun_out/prof_${T}_tb_trace.log; exit 1; }
bash tools/prof_cfg.sh ${T}_kaggle kaggle || { tail -n 20 gpurun_out/prof_${T}_kaggle_trace.log; exit 1; }
EXTRA="--batch-per-gpu 128 --mode sgd --gather-batch 0 --steps 200 --warmup 20" bash tools/prof_cfg.sh ${T}_c3 kaggle || { tail -n 20 gpurun_out/prof_${T}_c3_trace.log; exit 1; }
cd $R
for c in tb kaggle c3; do
  python3 tools/prof_summary.py gpurun_out/prof_${T}_$c gpurun_out/${T}_$c > gpurun_out/${T}_${c}_prof.txt && head -n 6 gpurun_out/${T}_${c}_prof.txt
done
