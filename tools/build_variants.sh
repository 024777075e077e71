#!/bin/bash
# Build experiment variants of libsva.so for in-process A/B (tools/ab_paths.py):
#   tools/build_variants.sh name1 "kPfH8=28 kPfV8=8" name2 "kWtahPfBwd=6" ...
# Each variant is built from a scratch copy of stereovisionarray_amd/csrc
# (build/var_<name>/src) whose sva_tuning.h has the named constexpr constants
# rewritten; product translation units carry no experiment switches.  A value
# may also be a whole replacement file: name "@path/to/tuning.h".
# Output: $AB_DIR/libsva_<name>.so, default ab_libs/ (gpurun-ignored: set
# AB_DIR=ab_run for libraries a GPU run loads).  The product libsva.so is untouched.
set -eu
cd "$(dirname "$0")/.."
AB=${AB_DIR:-ab_libs}
mkdir -p "$AB"
while [ $# -ge 2 ]; do
  name=$1 spec=$2; shift 2
  src=build/var_$name/src
  rm -rf "$src"; mkdir -p "$src"
  cp stereovisionarray_amd/csrc/* "$src"/
  if [ "${spec#@}" != "$spec" ]; then
    cp "${spec#@}" "$src/sva_tuning.h"
  else
    for kv in $spec; do
      k=${kv%%=*} v=${kv#*=}
      grep -q "\b$k = " "$src/sva_tuning.h" || { echo "unknown tuning constant $k"; exit 2; }
      sed -i -E "s/\b($k) = [^,;]+/\1 = $v/" "$src/sva_tuning.h"
    done
  fi
  make -s -j8 -C "$src" BUILD="$PWD/build/var_$name/obj" OUT="$PWD/$AB/libsva_$name.so" \
       INC="$PWD/include"
  echo "built $AB/libsva_$name.so ($spec)"
done
