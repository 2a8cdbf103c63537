#!/bin/bash
# Build an A/B variant of libbopx.so from a patched COPY of csrc (the product
# sources stay free of experiment switches):
#   bash tools/mkvar_patch.sh NAME "SED_SCRIPT" ["-DFLAG=VALUE ..."]
#   -> bop_toolkit_amd/lib/variants/NAME.so
# SED_SCRIPT is applied to kern_vsd.hip, kern_pose.hip and raster.h of the copy.
# REV=<git revision> patches that revision's sources instead of the working tree.
set -e
cd "$(dirname "$0")/../bop_toolkit_amd"
src=csrc_var_$1
rm -rf "$src"; mkdir -p "$src"
if [ -n "$REV" ]; then
  (cd .. && git archive "$REV" bop_toolkit_amd/csrc) | tar -x -C "$src" --strip-components=2
else
  cp csrc/*.hip csrc/*.h csrc/*.cpp csrc/Makefile "$src"/
fi
if [ -n "$2" ]; then sed -i -e "$2" "$src"/kern_vsd.hip "$src"/kern_pose.hip "$src"/raster.h; fi
make -s -j8 -C "$src" BUILD=build OUT=../lib/variants/$1.so IO_OUT=../lib/variants/io_unused.so EXTRA="$3" ../lib/variants/$1.so
rm -rf "$src"
