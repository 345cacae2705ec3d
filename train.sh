#!/bin/bash
# Reference train.sh launched main_dist.py in its single-process mode and dropped "$@" (missing
# line continuation). Here: one process per GPU over RCCL, args forwarded.
NGPUS=${NGPUS:-$(python3 -c "import torch; print(max(torch.cuda.device_count(), 1))")}
python3 -m torch.distributed.run --standalone --nproc-per-node "$NGPUS" main_dist.py \
  --batch_size 1024 \
  --output_dir ./test \
  --workers 16 \
  "$@"
