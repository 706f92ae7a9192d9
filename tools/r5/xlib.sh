# Fast experiment library: recompile only the given source with extra -D flags and link it with
# the product build's other objects (mli_nerf_amd/csrc/build/*.o).
#   bash tools/r5/xlib.sh <name> <source.hip> [flags...]  ->  xlib/<name>.so
# XSRC=<path> compiles that file in place of mli_nerf_amd/csrc/<source.hip> (e.g. an older
# revision from git show, for a baseline).
set -e
NAME=$1; SRC=$2; shift 2
B=mli_nerf_amd/csrc/build
mkdir -p xlib/obj_$NAME
H=$(python -c "from mli_nerf_amd import build as b; print(b.source_hash())")
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -I include -I mli_nerf_amd/csrc \
  -DMLI_SOURCE_HASH="\"$H\"" "$@" -x hip -c ${XSRC:-mli_nerf_amd/csrc/$SRC} -o xlib/obj_$NAME/${SRC%.hip}.o
# params.hip carries the embedded source hash: rebuilt with the tree's current hash
[ "$SRC" = params.hip ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -I include \
  -I mli_nerf_amd/csrc -DMLI_SOURCE_HASH="\"$H\"" -c mli_nerf_amd/csrc/params.hip -o xlib/obj_$NAME/params.o
OBJS=""
for o in $(python -c "from mli_nerf_amd import build as b; print(' '.join('$B/' + x[:-4] + '.o' for x in b.SOURCES))"); do
  b=$(basename $o)
  if [ "$b" = "${SRC%.hip}.o" ] || [ "$b" = params.o ]; then OBJS="$OBJS xlib/obj_$NAME/$b"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o xlib/$NAME.so $OBJS
echo xlib/$NAME.so
