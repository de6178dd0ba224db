#!/bin/bash
# build libfsg.so with extra defines into fluvio_amd/DIR: build_variant.sh DIR "-DFOO -DBAR"
set -e
cd "$(dirname "$0")/../fluvio_amd/csrc"
make -s -j8 OUT=../$1 EXTRA="$2" ../$1/libfsg.so
