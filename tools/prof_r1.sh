set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --cpu-baseline 0 --gather-iters 20"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1_trace -o tb --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_r1_trace.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_r1_fetch -o tb --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_r1_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_r1_write -o tb --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_r1_write.log 2>&1
