#!/bin/bash
# Experiment variant of libsqr (never the shipped library): sqr_conv3.hip rebuilt with
# -DSQR_EXPERIMENTS (forced tile configurations SQR_D3_CFG / SQR_S2F_CFG, ablation bits SQR_EXP) and,
# with "stamps" as the first argument, the per-workgroup SQR_STAMPS timeline too.  Linked with the
# regular objects (make first).  Output: tools/exp_lib/libsqr.so or tools/exp_stamps_lib/libsqr.so
set -euo pipefail
cd "$(dirname "$0")/.."
make -C sq-recovery_amd/csrc -j8 >/dev/null
defs="-DSQR_EXPERIMENTS"
out=tools/exp_lib
if [ "${1:-}" = "stamps" ]; then
  defs="$defs -DSQR_STAMPS -DSQR_STAMP_MAXWG=8192"
  out=tools/exp_stamps_lib
fi
mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics $defs \
  -c sq-recovery_amd/csrc/sqr_conv3.hip -o $out/sqr_conv3.o
objs=$(ls build/obj/*.o | grep -v sqr_conv3.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o $out/libsqr.so $objs $out/sqr_conv3.o
rm -f $out/sqr_conv3.o
