# rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of tools/bench_rowwise.py
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS="--shape ${SHAPE:-tb} --iters 20"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rw_trace -o tb --output-format csv -- python3 $R/tools/bench_rowwise.py $ARGS > $R/gpurun_out/prof_rw_trace.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_rw_fetch -o tb --output-format csv -- python3 $R/tools/bench_rowwise.py $ARGS > $R/gpurun_out/prof_rw_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_rw_write -o tb --output-format csv -- python3 $R/tools/bench_rowwise.py $ARGS > $R/gpurun_out/prof_rw_write.log 2>&1
