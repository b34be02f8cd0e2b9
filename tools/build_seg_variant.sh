# build lib_var/<name>/libf110qp.so with the segmented lane kernel (lane_seg_inst.hip) recompiled
# from <src dir> under extra -D flags (measurement only, F110QP_LIB selects it). Usage from the
# repo root: tools/build_seg_variant.sh <name> <src dir with lane_seg_kernel.h> <flags...>
set -e
name=$1; src=$2; shift 2
cd f110-mpc_amd
d=build_var/$name; mkdir -p $d lib_var/$name
cp csrc/lane_seg_inst.hip csrc/f110qp_kernels.h $d/
cp $src/lane_seg_kernel.h $d/
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -I$d $* -c $d/lane_seg_inst.hip -o $d/lane_seg_inst.o
others=$(ls build_obj/*.o | grep -v "build_obj/lane_seg_inst.o" | grep -v "build_obj/f110qp_api_test.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_var/$name/libf110qp.so $others $d/lane_seg_inst.o
echo built lib_var/$name/libf110qp.so
