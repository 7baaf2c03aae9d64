#!/bin/bash
# Host AddressSanitizer + UBSan build of the native planner / JIT code generator, run on random
# circuits (tools/native_fuzz.cpp).  CPU only: GPU ASan / XNACK runs are not available on the pool.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p build/asan
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
g++ -std=c++17 -O1 -g $SAN -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
    tools/native_fuzz.cpp qfedx_amd/csrc/planner.cpp qfedx_amd/csrc/jit.cpp \
    -L/opt/rocm/lib -lhiprtc -lamdhip64 -Wl,-rpath,/opt/rocm/lib -o build/asan/native_fuzz
ASAN_OPTIONS=detect_leaks=1 ./build/asan/native_fuzz "${1:-300}"
