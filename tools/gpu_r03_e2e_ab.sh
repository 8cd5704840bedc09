# End-to-end A/B on one box: the cmsbwt CLI on the bench workload's FASTA
# files, with and without the collection upload overlapping the index build
# (CMSBWT_OVERLAP_UPLOAD), interleaved; then the 2-rank bench rehearsal
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
W=$(mktemp -d /tmp/e2eab_XXXX)
cms-bwt_amd/build/gen_synth 10000000 1000 0.001 4 $W/w
for i in 1 2 3 4 5; do
  for ov in 1 0; do
    s=$(date +%s.%N)
    CMSBWT_OVERLAP_UPLOAD=$ov timeout -k 10 60 cms-bwt_amd/build/cmsbwt -r -v -o $W/out $W/w.list 2> $W/err > /dev/null
    e=$(date +%s.%N)
    echo "overlap=$ov wall=$(echo "$e - $s" | bc) $(tail -1 $W/err)"
  done
done | tee gpurun_out/e2e_ab.txt
sha256sum $W/out.rl_bwt | cut -c1-16
rm -rf $W
bash tools/gpu_r03_bench2.sh
