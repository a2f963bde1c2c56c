# Build a libkcnn variant that differs from libkcnn.so only in one source's
# compile flags:
#   experiments/build_src_var.sh NAME SRC "-DFLAG ..."  -> kaldi-cnn_amd/libkcnn_NAME.so
# (SRC relative to kaldi-cnn_amd/src, e.g. kaldi-lite/cu-gemm-f16x3.hip)
set -e
cd "$(dirname "$0")/../kaldi-cnn_amd"
make -s -j8 libkcnn.so
mkdir -p build/var
obj=build/$(dirname $2)/$(basename $2 .hip).o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../include -Isrc -I/opt/rocm/include \
  --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize $3 -c src/$2 -o build/var/$1.o
objs=$(ls build/{capi,cnslmat,kaldi-lite,nnet0,nnet2}/*.o | grep -v "^$obj\$")
/opt/rocm/bin/hipcc $objs build/var/$1.o -shared -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocblas -lamdhip64 -o libkcnn_$1.so
echo built libkcnn_$1.so
