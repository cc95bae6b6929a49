# Build a variant of libdcx.so with extra compile flags into distilcodec_nabeel_amd/<name>.so
# (select it at run time with DCX_LIB=...).  Usage: bash tools/build_variant.sh NAME "-DFLAG ..."
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
B=$R/distilcodec_nabeel_amd/csrc/build_$NAME
mkdir -p $B
CXX="/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -Wno-unused-value --offload-arch=gfx950 $FLAGS"
cd $R/distilcodec_nabeel_amd/csrc
$CXX -c dcx_conv.hip -o $B/dcx_conv.o &
$CXX -c dcx_misc.hip -o $B/dcx_misc.o &
$CXX -c dcx_resblock.hip -o $B/dcx_resblock.o &
$CXX -x hip -c dcx_api.cpp -o $B/dcx_api.o &
g++ -O3 -fPIC -std=c++17 -c dcx_mp3.cpp -o $B/dcx_mp3.o &
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $R/distilcodec_nabeel_amd/$NAME.so $B/dcx_conv.o $B/dcx_misc.o $B/dcx_resblock.o $B/dcx_mp3.o $B/dcx_api.o
echo built $R/distilcodec_nabeel_amd/$NAME.so
