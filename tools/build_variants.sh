#!/bin/bash
# Build tuning variants of libsrs_amd.so into simd-radix-sort_amd/lib/variants/<name>/.
# usage: tools/build_variants.sh name:"-DFOO=1 -DBAR=2" ...
set -e
cd "$(dirname "$0")/../simd-radix-sort_amd"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=lib/variants/$name; rm -rf $out build/v_$name; mkdir -p $out build/v_$name
  pids=()
  for f in srs_kernels srs_api srs_shard; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags \
      -Rpass-analysis=kernel-resource-usage -c csrc/$f.hip -o build/v_$name/$f.o 2> build/v_$name/$f.remarks &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || { echo "FAILED $name"; exit 1; }; done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libsrs_amd.so build/v_$name/*.o -ldl -Wl,-rpath,/opt/rocm/lib
  echo "built $name ($flags)"
done
