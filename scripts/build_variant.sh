# Build an in-tree variant of the HIP library with extra -D flags on gs_blend.hip (A/B experiments):
#   bash scripts/build_variant.sh NAME -DFOO=1 ...   -> gaussiansplatting_amd/lib/libgs_NAME.so
set -e
name=$1; shift
mkdir -p build/var_$name
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Iinclude -Igaussiansplatting_amd/csrc"
for s in gs_sort gs_segsort gs_raster gs_blend gs_chain gs_density gs_optim gs_loss gs_membw; do
  /opt/rocm/bin/hipcc $F "$@" -c gaussiansplatting_amd/csrc/$s.hip -o build/var_$name/$s.o &
done
/opt/rocm/bin/hipcc $F "$@" -x hip -c gaussiansplatting_amd/csrc/gs_capi.cpp -o build/var_$name/gs_capi.o &
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -ffp-contract=off -c gaussiansplatting_amd/csrc/gs_io.cpp -o build/var_$name/gs_io.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o gaussiansplatting_amd/lib/libgs_$name.so build/var_$name/*.o
echo built gaussiansplatting_amd/lib/libgs_$name.so
