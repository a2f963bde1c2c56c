# r05: the fused Conv -> Maxpool(2x1x4) forward at 601 frames, G = 96:
# repeated calls against their own majority and fused vs unfused, for the
# current library, its inline-asm-split variant and the r04 library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05f; mkdir -p $O
for v in cur asm r04; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $v != cur ] && L=$PWD/kaldi-cnn_amd/libkcnn_$v.so
  for s in halfB_G96_2x1x4 pc2_G96 c2; do
    STACK=$s REPS=30 KCNN_LIB=$L timeout -k 10 200 python experiments/diag_fused_pool.py >> $O/diag_$v.txt 2>&1 || { echo "diag $v $s rc $?"; cat $O/diag_$v.txt | tail -5; exit 4; }
  done
  echo "== $v"; grep -v amdgpu.ids $O/diag_$v.txt
done
