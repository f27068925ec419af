N=motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native
for B in 4096 32768 65536 131072; do timeout -k 10 100 python tools/ablate.py $B f64 "$N/libikgrasp.so" 2>&1 | grep "B="; done
for B in 32768 65536 131072 262144; do timeout -k 10 100 python tools/ablate.py $B f32 "$N/libikgrasp.so" 2>&1 | grep "B="; done
