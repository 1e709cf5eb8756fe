set -eo pipefail
cd $GRAFT_REPO_ROOT
for v in libspecdec.so libspecdec_w8s16.so libspecdec_w4s16.so libspecdec_w2s32.so; do
  echo "== $v" >> gpurun_out/thresh_ab.log
  SPECDEC_LIB=$v timeout -k 10 120 python scripts/debug/thresh_rows.py 2>&1 | tail -1 >> gpurun_out/thresh_ab.log
  SPECDEC_LIB=$v timeout -k 10 120 python scripts/debug/thresh_time.py 2>&1 | grep rows >> gpurun_out/thresh_ab.log
done
