#!/bin/bash
# Debug variant of the library with every exact-smpl array index checked (LZ_SMPL_CHECK in
# csrc/smpl.hip): tools/ablib/chk.so, the other objects from the normal build.  Use it with
# LZ77SSS_LIB=tools/ablib/chk.so; violations print "[lz77sss] smpl check ... FAIL site ...".
set -e
cd "$(dirname "$0")/../lz77-sss_amd"
make -s -j8
mkdir -p ../tools/ablib build/chk
/opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function \
    -fvisibility=hidden -DLZ_SMPL_CHECK -c csrc/smpl.hip -o build/chk/smpl.hip.o
objs=$(ls build/*.o | grep -v '/smpl.hip.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/chk/smpl.hip.o -o ../tools/ablib/chk.so
echo "built tools/ablib/chk.so"
