# The bench's multi-rank path on a one-GPU box: 2 and 4 ranks sharing the GPU,
# gloo collectives on host copies (IKG_BENCH_BACKEND=gloo).  The measured
# configuration (one rank per GPU over RCCL) runs on the driver's 8-GPU node.
set -o pipefail
mkdir -p gpurun_out/multirank
for n in 2 4; do
  IKG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 1 \
    > gpurun_out/multirank/n$n.json 2> gpurun_out/multirank/n$n.err || exit $?
  IKG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29510 + n)) bench.py --gpus $n --steps 3 --warmup 1 --batch 512 --multistart 64 \
    > gpurun_out/multirank/ms_n$n.json 2>> gpurun_out/multirank/n$n.err || exit $?
done
cut -c1-400 gpurun_out/multirank/*.json
