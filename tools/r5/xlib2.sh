# Experiment library from several replaced sources: each listed source is compiled from <srcdir>
# (its own headers first -- e.g. an older revision's mlp_core.h / common.h from git show) and
# linked with the product build's other objects.
#   [XFLAGS="-D..."] bash tools/r5/xlib2.sh <name> <srcdir> <a.hip> [b.hip ...]  ->  xlib/<name>.so
set -e
NAME=$1; DIR=$2; shift 2
B=mli_nerf_amd/csrc/build
mkdir -p xlib/obj_$NAME
H=$(python -c "from mli_nerf_amd import build as b; print(b.source_hash())")
CXX="/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -I include -I mli_nerf_amd/csrc"
for SRC in "$@"; do
  $CXX $XFLAGS -DMLI_SOURCE_HASH="\"$H\"" -c $DIR/$SRC -o xlib/obj_$NAME/${SRC%.hip}.o &
done
$CXX -DMLI_SOURCE_HASH="\"$H\"" -c mli_nerf_amd/csrc/params.hip -o xlib/obj_$NAME/params.o &
wait
OBJS=""
for o in $(python -c "from mli_nerf_amd import build as b; print(' '.join('$B/' + x[:-4] + '.o' for x in b.SOURCES))"); do
  b=$(basename $o)
  if [ -f xlib/obj_$NAME/$b ]; then OBJS="$OBJS xlib/obj_$NAME/$b"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o xlib/$NAME.so $OBJS
echo xlib/$NAME.so
