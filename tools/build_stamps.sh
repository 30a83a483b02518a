#!/bin/bash
# SQR_STAMPS variant of libsqr for tools/conv_stamps.py: sqr_conv3.hip rebuilt with per-workgroup
# wall-clock stamps, linked with the regular objects (make first).  Output: tools/stamps_lib/libsqr.so
set -euo pipefail
cd "$(dirname "$0")/.."
make -C sq-recovery_amd/csrc -j8 >/dev/null
mkdir -p tools/stamps_lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -DSQR_STAMPS -DSQR_STAMP_MAXWG=8192 \
  -c sq-recovery_amd/csrc/sqr_conv3.hip -o tools/stamps_lib/sqr_conv3.o
objs=$(ls build/obj/*.o | grep -v sqr_conv3.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o tools/stamps_lib/libsqr.so $objs tools/stamps_lib/sqr_conv3.o
rm -f tools/stamps_lib/sqr_conv3.o
