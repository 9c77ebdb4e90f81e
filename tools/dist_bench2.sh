# bench.py at world 2 on the box's one GPU (gloo): the N>1 code path of the driver's
# scaling run (RCCL there), with short recon/q-dq settings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline --recon-iters 30
