# Error events of repeated frame forwards (experiments/diag_det2.py) on a few
# shapes, default library.
set -o pipefail
for S in halfB c2 k4g64 g40; do
  SHAPE=$S KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn.so REPS=${REPS:-60} timeout -k 10 150 python experiments/diag_det2.py || exit 3
done
