# r06 first call: the new parity tests (c5 at 4096 frames, the adversarial
# C3 -> P2, the GEMM's beta-1 spread case), then bench lines c2 / c5 / nnet
# and a same-box A/B against the r05 library on c2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r06a}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_full.py tests/test_gpu_gemm.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|Error|passed|failed" $O/pytest.txt | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
for i in 1 2; do for lib in r05 new; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $lib = r05 ] && L=$PWD/kaldi-cnn_amd/libkcnn_r05.so
  KCNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/ab_${lib}_$i.json > $O/ab_${lib}_$i.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/ab_${lib}_$i.json'));print('$lib', d['value'], d['ms_per_step'], d['profiled_ms_per_step'])"
done; done
for cfg in c5 nnet; do
timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --json-out $O/$cfg.json > $O/$cfg.log 2>&1 || exit 5
python -c "
import json;d=json.load(open('$O/$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['profiled_ms_per_step'], d['roofline']['frac'], d['roofline']['peak'], d['conv']['f16x3_igemm_calls_per_step'])"
done
