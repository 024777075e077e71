#!/bin/bash
# Build experiment variants of libsva.so for in-process A/B (tools/ab_paths.py):
#   tools/build_variants.sh name1 "-DFOO=1 -DBAR=2" name2 "-DBAZ=3" ...
# Output: ab_libs/libsva_<name>.so (the product libsva.so is untouched).
set -eu
cd "$(dirname "$0")/.."
mkdir -p ab_libs
while [ $# -ge 2 ]; do
  name=$1 flags=$2; shift 2
  make -s -j8 -C stereovisionarray_amd/csrc BUILD=../../build/var_$name \
       OUT=../../ab_libs/libsva_$name.so EXTRA="$flags"
  echo "built ab_libs/libsva_$name.so ($flags)"
done
