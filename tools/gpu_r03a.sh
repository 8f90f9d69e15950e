#!/bin/bash
# Round 3, first GPU pass: the new reply/batcher/placement/RCCL-self tests,
# the reply checks added to the parity suite, then the full-size C4/C5 tests.
set -o pipefail
O=gpurun_out/r03a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_replication.py tests/test_group.py tests/test_batcher.py \
  "tests/test_gpu_parity.py::test_mixed_stream_vs_oracle" \
  "tests/test_gpu_parity.py::test_mixed_stream_hot_buckets_block_fold" \
  "tests/test_gpu_parity.py::test_mixed_hot_adversarial_all_fold_kinds" \
  "tests/test_gpu_parity.py::test_small_batches_one_launch_vs_large_path_and_oracle" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 ./tools/take_load 16 2000 20 100000 2 0.01 > $O/take_load.jsonl 2> $O/take_load.err || exit 1
timeout -k 10 120 ./tools/take_load 64 1000 20 100000 2 0.01 >> $O/take_load.jsonl 2>> $O/take_load.err || exit 1
timeout -k 10 120 ./tools/take_load 64 1000 20 100000 0 >> $O/take_load.jsonl 2>> $O/take_load.err || exit 1
cat $O/take_load.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread \
  "tests/test_fullsize.py::test_c4_shard_full_size_rccl_exchange" \
  "tests/test_fullsize.py::test_c5_full_size_anti_entropy_vs_go_merge" \
  > $O/full.log 2>&1 || { tail -40 $O/full.log; exit 1; }
tail -3 $O/full.log
