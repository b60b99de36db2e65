#!/bin/bash
# Build libsrs_amd.so from a git revision's sources into
# simd-radix-sort_amd/lib/variants/<name>/ (A/B timing against the work tree).
# usage: tools/build_rev_variant.sh <name> <rev> [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2; shift 2
src=$(mktemp -d)
mkdir -p $src/include $src/pkg/csrc
for f in srs_kernels.hip srs_api.hip srs_common.h srs_kernels.h; do
  git show $rev:simd-radix-sort_amd/csrc/$f > $src/pkg/csrc/$f
done
git show $rev:include/srs_c_api.h > $src/include/srs_c_api.h
out=simd-radix-sort_amd/lib/variants/$name; mkdir -p $out
for f in srs_kernels srs_api; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics "$@" \
    -c $src/pkg/csrc/$f.hip -o $src/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libsrs_amd.so $src/*.o -Wl,-rpath,/opt/rocm/lib
rm -rf $src
echo "built $name from $rev"
