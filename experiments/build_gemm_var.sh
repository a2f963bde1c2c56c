# Build libkcnn variants that differ only in cu-gemm-x6.hip compile flags:
#   scripts/build_gemm_var.sh NAME "-DFLAG=..."   -> kaldi-cnn_amd/libkcnn_NAME.so
set -e
cd "$(dirname "$0")/../kaldi-cnn_amd"
make -s -j8 libkcnn.so
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../include -Isrc -I/opt/rocm/include \
  --offload-arch=gfx950 -munsafe-fp-atomics $2 -c src/kaldi-lite/cu-gemm-x6.hip -o build/var/gemm-$1.o
objs=$(ls build/{capi,cnslmat,kaldi-lite,nnet0,nnet2}/*.o | grep -v cu-gemm-x6.o)
/opt/rocm/bin/hipcc $objs build/var/gemm-$1.o -shared -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocblas -lamdhip64 -o libkcnn_$1.so
echo built libkcnn_$1.so
