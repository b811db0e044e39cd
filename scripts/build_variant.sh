#!/bin/bash
# A/B experiment builds: the product objects with ONE source replaced by a variant (a modified copy anywhere, or the
# product file under extra -D flags), linked to a variant library that scripts load through ICA_HIP_LIB (the product
# library is untouched).
#   bash scripts/build_variant.sh <name> <variant source> <product source it replaces> [-Dflags...]
#     -> scripts/variants/lib<name>.so
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; prod=$3; shift 3
C=imagecompression_adversarial_amd/csrc
mkdir -p scripts/variants
base=$(basename "$prod" .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-pass-failed -I$C "$@" -c "$src" -o scripts/variants/$base.$name.o
objs=""
for o in $C/*.o; do
  if [ "$(basename "$o" .o)" = "$base" ]; then objs="$objs scripts/variants/$base.$name.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/variants/lib$name.so $objs
echo scripts/variants/lib$name.so
