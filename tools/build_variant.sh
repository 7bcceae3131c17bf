#!/bin/bash
# Build an experimental libcfdj variant into build/<name>/libcfdj.so with extra HIP flags;
# select it at run time with CFDJ_LIB=build/<name>/libcfdj.so.
# usage: tools/build_variant.sh <name> "<extra flags>"
set -e
name=$1; shift
d=build/$name; mkdir -p $d
cd cfd_julia_amd/csrc
make -s -j8 OUT=../../$d/libcfdj.so OBJDIR=../../$d EXTRA="$*" ../../$d/libcfdj.so
