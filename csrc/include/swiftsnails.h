// swiftsnails.h — umbrella header of the native (C++) API, the counterpart of
// the reference's src/swiftsnails.h:8-17 (utils + core + framework in one
// include).  Host runtime (header-only, C++17, no GPU needed):
//
//   BinaryBuffer (buffer.h)          codec of the wire format and checkpoints
//   Config / global_config (config.h) `key: value`, `#`, `import`, first wins
//   Channel, ThreadPool, StateBarrier, SpinLock (channel.h)
//   HashFrag (hashfrag.h)            fragment -> node router, fmix64-exact
//   HostTable (host_table.h)         lock-striped CPU shard + text dump
//   Transfer, MetaMessage, Addr (transfer.h)  TCP request/response RPC
//   Master, Server, WorkerClient (cluster.h)  the three roles of a host job
//   Vec (vec.h), string helpers (string_util.h), data loaders (dataio.h)
//   ss::fmix64, ss::opt_apply (ss/hash.h, ss/optim.h)  shared with the HIP kernels
//
// GPU side: csrc/hip/worker.h (ss::GpuWorker: pull / push against one GPU's
// HBM table with async handles, compiled into _ss_hip with the kernels); the
// multi-GPU round engine (RCCL all-to-all-v rounds, pull-ahead) is driven from
// Python (swiftsnails_amd.parallel.PSEngine) over the same kernels.
#pragma once

#include "ss/hash.h"
#include "ss/optim.h"

#include "buffer.h"
#include "channel.h"
#include "cluster.h"
#include "config.h"
#include "dataio.h"
#include "hashfrag.h"
#include "host_table.h"
#include "string_util.h"
#include "transfer.h"
#include "vec.h"
