# duo layout with one wave per SIMD (AGPR claim) vs shared-SIMD placement vs pair
mkdir -p gpurun_out/r4d
timeout -k 10 200 python tools/layout_ab.py --variants 1,4 --sizes 4096,16384 --out gpurun_out/r4d/ab_wps1.json > gpurun_out/r4d/ab_wps1.log 2>&1
echo "ab rc=$?"
IKG_DUO_SHARED=1 timeout -k 10 200 python tools/layout_ab.py --variants 1,4 --sizes 4096 --dtypes f64 --out gpurun_out/r4d/ab_shared.json > gpurun_out/r4d/ab_shared.log 2>&1
echo "ab shared rc=$?"
