# Build a variant of libdgadv.so that differs only in dg_rec.hip's compile flags: the other
# translation units are the product's objects (lib/obj/).  Experiments only.
#   bash profiles/r02/build_rec_variant.sh <name> [-DFOO ...]   -> adjoint-ode-adaptivity_amd/lib/var_<name>.so
set -e
cd "$(dirname "$0")/../.."
PKG=adjoint-ode-adaptivity_amd
NAME=$1; shift
mkdir -p $PKG/lib/obj_var
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -I include "$@" -c -o $PKG/lib/obj_var/dg_rec_$NAME.o $PKG/csrc/dg_rec.hip
OBJS=$(ls $PKG/lib/obj/*.o | grep -v dg_rec.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/var_$NAME.so $OBJS $PKG/lib/obj_var/dg_rec_$NAME.o
echo "built $PKG/lib/var_$NAME.so"
