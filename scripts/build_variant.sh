#!/bin/bash
# Build an A/B variant of libusv.so with extra defines for the fast kernel:
#   scripts/build_variant.sh <name> -DUSV_XCD_REMAP=0 ...
# -> build_variants/<name>.so (same C ABI; select with USV_LIB_PATH).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
SRC=${VARIANT_SRC:-usv_sad_fast}   # which kernel file the defines apply to
C=unsynchronized_stereo_vision_proj325_amd/csrc
make -s -C $C
OUTD=${VARIANTS_DIR:-build_variants}; mkdir -p $OUTD
# VARIANT_FILE: compile this file in place of $C/$SRC.hip (e.g. an older revision from git show)
EXTRA=""
[ "$SRC" = usv_ssd_mfma ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form"  # as the Makefile's per-object flag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Iinclude -I$C -ffp-contract=off -DUSV_VARIANT_BUILD=1 $EXTRA "$@" \
    -c ${VARIANT_FILE:-$C/$SRC.hip} -o $OUTD/$name.var.o
# the C ABI object again with USV_VARIANT_BUILD: usv_version() of a variant says "variant build"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Iinclude -I$C -ffp-contract=off -DUSV_VARIANT_BUILD=1 \
    -c $C/usv_capi.hip -o $OUTD/$name.capi.o
objs=$(ls $C/build/*.o | grep -v "/$SRC.o" | grep -v "/usv_capi.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUTD/$name.so $OUTD/$name.var.o $OUTD/$name.capi.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f $OUTD/$name.var.o $OUTD/$name.capi.o
echo built $OUTD/$name.so
