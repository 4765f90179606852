# rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE + read-request-size passes (separate runs) of a short bench
# run for one config; summarise with: python tools/prof_summary.py gpurun_out/prof_<tag> profiles/r2_<tag>
# usage: bash tools/prof_cfg.sh <tag> <config>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1
CFG=$2
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS="--config $CFG --steps 20 --warmup 5 --cpu-baseline 0 --gather-iters 20 --mlp-iters 10 ${EXTRA:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_trace -o tb --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_${TAG}_trace.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${TAG}_fetch -o tb --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_${TAG}_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${TAG}_write -o tb --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_${TAG}_write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $R/gpurun_out/prof_${TAG}_rdreq -o tb --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_${TAG}_rdreq.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum -d $R/gpurun_out/prof_${TAG}_wrreq -o tb --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_${TAG}_wrreq.log 2>&1
