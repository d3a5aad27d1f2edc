set -e
mkdir -p gpurun_out/dbg
cd gpurun_out/dbg
export PYTHONPATH=$GRAFT_REPO_ROOT DNN_BACKEND=gloo OMP_NUM_THREADS=2 DNN_DEBUG_XGMI=1
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29801 $GRAFT_REPO_ROOT/tools/xgmi_reform_check.py > reform_keep.log 2>&1 || echo "rc=$?" >> reform_keep.log
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29802 $GRAFT_REPO_ROOT/tools/xgmi_reform_check.py --close-first > reform_close.log 2>&1 || echo "rc=$?" >> reform_close.log
ARGS="--epochs 3 --batch-size 32 --sync step-allreduce --train-samples 768 --test-samples 256 --device cuda --nb-proc 3 --check-sync"
timeout -k 10 200 python -m distributed_neural_network_amd.parallel.launch -n 3 $GRAFT_REPO_ROOT/data_parallelism_train.py $ARGS --drop-rank 1 --drop-at-epoch 1 --drop-at-step 2 > drop_xgmi.log 2>&1 || echo "rc=$?" >> drop_xgmi.log
