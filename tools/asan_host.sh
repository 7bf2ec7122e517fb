#!/bin/bash
# Host-side AddressSanitizer run of the CPU test suite: a copy of the tracked tree in /tmp, the
# library rebuilt with -fsanitize=address on the host code only (-Xarch_host; GPU code is not
# instrumented), the suite run with the ASan runtime preloaded into Python.  Not for the GPU box.
#   bash tools/asan_host.sh            (about 10 minutes on 8 cores)
set -e
SRC=$(cd "$(dirname "$0")/.." && pwd)
DST=${ASAN_TREE:-/tmp/asanrepo}
rm -rf "$DST" && mkdir -p "$DST"
(cd "$SRC" && git ls-files | grep -v '^profiles/' | tar -cf - -T -) | tar -xf - -C "$DST"
make -s -j8 -C "$DST/circulantpreconditioner_amd/csrc" \
  EXTRA_FLAGS="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer" \
  LDFLAGS="-shared -fsanitize=address -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib"
make -s -C "$DST/oracle"
ASANLIB=$(/opt/rocm/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
cd "$DST"
# the bench self-launch tests spawn interpreters the preload would also instrument; the reference
# caller link test would need -fsanitize=address on its own link line
ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:replace_intrin=0:detect_odr_violation=0 LD_PRELOAD=$ASANLIB \
  python -m pytest tests/ -q -m "not gpu" -p no:cacheprovider --deselect tests/test_bench_cpu.py -k "not compiles_unchanged"
