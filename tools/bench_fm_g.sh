#!/usr/bin/env bash
# FM / word2vec throughput vs table lane-group size (SS_TABLE_G)
set -u
for g in 16 4; do
  echo "=== FM G=$g"
  SS_TABLE_G=$g timeout -k 10 300 python -m swiftsnails_amd.launch --config configs/fm_10b.conf --steps 30 --warmup 5 --set num_features=1000000000 --set table_stats=0 2>&1 | grep '^{' | cut -c1-200
done
echo "=== w2v"
timeout -k 10 300 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 30 --warmup 5 --set server_ranks=all --set worker_ranks=all --set table_stats=0 2>&1 | grep '^{' | cut -c1-200
