#!/bin/bash
# Host-only AddressSanitizer + UBSan build of the kernel library's planning code and the harness
# (device code compiled as usual at -O3, uninstrumented: the -O1 device build of the halo wgrad
# DMA issue hits a gfx950 backend register-class error; nothing is launched). CPU only.
set -e
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT=${SAN_OUT:-/tmp/pca_sanitize}
mkdir -p "$OUT"
CSRC="$ROOT/pytorch_cifar_amd/csrc"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="-x hip --offload-arch=gfx950 -O3 -Xarch_host -O1 -Xarch_host -g -std=c++17 -fno-omit-frame-pointer \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
  -I$CSRC -Wno-unused-result -Wno-unused-command-line-argument"
objs=()
for f in conv_mfma conv_halo conv3x3_c64 conv3x3_hx conv1x1_nk stem batchnorm; do
  $HIPCC $FLAGS -c "$CSRC/$f.hip" -o "$OUT/$f.o" &
  objs+=("$OUT/$f.o")
done
wait
$HIPCC -x hip --offload-arch=gfx950 -O1 -g -std=c++17 -Xarch_host -fsanitize=address \
  -Xarch_host -fsanitize=undefined -I"$CSRC" -c "$ROOT/tools/sanitize/host_plan_check.cpp" -o "$OUT/main.o"
$HIPCC -fno-gpu-sanitize -fsanitize=address -fsanitize=undefined "$OUT/main.o" "${objs[@]}" -o "$OUT/host_plan_check" \
  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_plan_check"
