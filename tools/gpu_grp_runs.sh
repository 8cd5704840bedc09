set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/grp
for v in 1 0; do
  CMSBWT_GRP_RUNS=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/grp/v$v -o kt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/grp/v$v.log 2>&1
  echo "v$v $(tail -1 gpurun_out/grp/v$v.log | cut -c1-200)"
  python3 tools/kstats.py gpurun_out/grp/v$v/kt_kernel_stats.csv | grep -E "grp_seg|run_bin|k_finalize" 
  rm -f gpurun_out/grp/v$v/kt_kernel_trace.csv
done
