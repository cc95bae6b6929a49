# Build a variant of libdcx.so whose dcx_resblock.hip is compiled with extra flags (the other objects
# are the in-tree build's) into distilcodec_nabeel_amd/<name>.so; select it with DCX_LIB=...
# Usage: bash tools/build_rp_variant.sh NAME "-DFLAG ..."
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
C=$R/distilcodec_nabeel_amd/csrc
B=$C/build_$NAME
mkdir -p $B
make -C $C -s >/dev/null
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -Wno-unused-value --offload-arch=gfx950 $FLAGS -c $C/dcx_resblock.hip -o $B/dcx_resblock.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $R/distilcodec_nabeel_amd/$NAME.so $C/build/dcx_conv.o $C/build/dcx_misc.o $B/dcx_resblock.o $C/build/dcx_mp3.o $C/build/dcx_api.o
echo built $R/distilcodec_nabeel_amd/$NAME.so
