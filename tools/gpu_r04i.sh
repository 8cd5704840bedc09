# Round 4, box I: HBM traffic of the merge-tail kernels (FETCH_SIZE and
# WRITE_SIZE passes, one rocprofv3 run each) on one bench step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/mt; rm -rf $OUT; mkdir -p $OUT
B1="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check"
RX="k_finalize|k_scatter_heads|k_ranks_slot|k_nhr_rank|k_nhr_rec|k_dbl_keys|k_dbl_rank|k_grp_seg|k_el_wr_emit|k_el_wr_count|k_item_fill64|k_wr_records|k_win_cross|radix_sort_onesweep_iteration"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $grp --kernel-include-regex "$RX" -d $OUT/p$i -o p$i --output-format csv -- $B1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_main.py $OUT > $OUT/pmc_main.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/mt/pmc_main.json"))
for k, v in sorted(d.items()):
    f, w = v.get("FETCH_SIZE", 0), v.get("WRITE_SIZE", 0)
    print(f"{k[:60]:60s} fetch {f/1024/1024:8.3f} GiB  write {w/1024/1024:8.3f} GiB  hit {v.get('TCC_HIT_sum',0):.3e} miss {v.get('TCC_MISS_sum',0):.3e}")
PY
