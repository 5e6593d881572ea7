# Build an experimental variant of the product library for an A/B run:
#   tools/build_variant.sh NAME -DFLAG ...   ->  lego-loam-bor_amd/lego_amd/liblego_frontend_NAME.so
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result -Wno-unused-value"
for s in lego_kernels.hip lego_frontend.hip lego_s2m.hip lego_mapper.hip lego_config.cpp; do
  /opt/rocm/bin/hipcc $F "$@" -c "$R/lego-loam-bor_amd/csrc/$s" -o "$T/$s.o" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "$T"/*.o -o "$R/lego-loam-bor_amd/lego_amd/liblego_frontend_$NAME.so"
rm -rf "$T"
echo "built liblego_frontend_$NAME.so"
