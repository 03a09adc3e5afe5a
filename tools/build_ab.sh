#!/bin/bash
# Builds an A/B variant of libfm3d.so: tools/build_ab.sh NAME "EXTRA HIPCC FLAGS"
# -> 3dfeaturematcher_amd/_ab/libfm3d_NAME.so (objects in _ab/obj_NAME); run with tools/ab.sh.
set -e
NAME=$1; EXTRA=$2
cd "$(dirname "$0")/../3dfeaturematcher_amd/csrc"
make -s -j8 OUT=../_ab/libfm3d_$NAME.so OBJDIR=../_ab/obj_$NAME EXTRA="$EXTRA" ../_ab/libfm3d_$NAME.so
