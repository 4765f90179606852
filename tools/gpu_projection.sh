# The 1 -> 8 GPU projection inputs: per-rank step time of rank 0 of an N-rank run on
# one GPU (bench.py --emulate-ranks N: the other ranks' maxima and payloads precomputed from their
# own slices, the two all-gathers replaced by resident buffers), TB weak (2048 per rank) and strong
# (2048 global, config 5) at N = 2/4/8, Kaggle config 4 (512 global) at N = 2/4, and a rocprofv3
# kernel trace of the TB N = 8 weak line. usage: bash tools/gpu_projection.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=$1
cd $R && mkdir -p gpurun_out
E="--steps 100 --warmup 10"
bash tools/gpu_run.sh $T \
  "bench=tbw2=--emulate-ranks 2 $E" "bench=tbw4=--emulate-ranks 4 $E" "bench=tbw8=--emulate-ranks 8 $E" \
  "bench=tbs2=--emulate-ranks 2 --scaling strong $E" "bench=tbs4=--emulate-ranks 4 --scaling strong $E" \
  "bench=tbs8=--emulate-ranks 8 --scaling strong $E" \
  "bench=kgs2=--config kaggle --emulate-ranks 2 --scaling strong --batch-per-gpu 512 $E" \
  "bench=kgs4=--config kaggle --emulate-ranks 4 --scaling strong --batch-per-gpu 512 $E" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_tbw8 -o r --output-format csv -- \
  python3 $R/bench.py --emulate-ranks 8 $E > $R/gpurun_out/${T}_prof_tbw8.log 2>&1 || { tail -20 $R/gpurun_out/${T}_prof_tbw8.log; exit 1; }
python3 $R/tools/kmedian.py $R/gpurun_out/prof_${T}_tbw8 > $R/gpurun_out/${T}_tbw8_kmedian.txt && cat $R/gpurun_out/${T}_tbw8_kmedian.txt
