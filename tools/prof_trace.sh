# rocprofv3 kernel trace of a short bench run: prints per-kernel average durations.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-trace}
CFG=${2:-terabyte}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o tb --output-format csv -- python3 $R/bench.py --config $CFG --steps 50 --warmup 10 --cpu-baseline 0 --gather-batch 0 > $R/gpurun_out/prof_$TAG.log 2>&1
