set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "coalesce or dp_ or parity" > gpurun_out/i1_tests.log 2>&1 || { tail -n 30 gpurun_out/i1_tests.log; exit 1; }
tail -n 1 gpurun_out/i1_tests.log
timeout -k 10 120 python tools/diag_coalesce.py terabyte > gpurun_out/i1_diag_tb.log 2>&1 || { tail gpurun_out/i1_diag_tb.log; exit 1; }
timeout -k 10 120 python tools/diag_coalesce.py kaggle > gpurun_out/i1_diag_kaggle.log 2>&1 || exit 1
cat gpurun_out/i1_diag_tb.log
bash tools/prof_cfg.sh i1_tb terabyte && python tools/prof_summary.py gpurun_out/prof_i1_tb profiles/r2b_tb > /dev/null && grep -o '"k_coalesce_p1[^}]*}' profiles/r2b_tb_summary.json
