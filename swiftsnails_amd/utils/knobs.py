"""Registry of the ``SS_*`` environment knobs.

Every environment variable the package, its kernels' launchers or the tools
read is listed here with its default, where it is read and what measuring it
showed; ``tests/test_knobs.py`` fails when a new one appears in the sources
without an entry (or an entry outlives its code).  Defaults are the measured
best; the experiment knobs keep alternatives that measured slower reachable
for re-measurement on other hardware.

    python -m swiftsnails_amd.utils.knobs        # print the table
"""
from __future__ import annotations

from typing import NamedTuple


class Knob(NamedTuple):
    default: str
    where: str
    kind: str  # "ops" | "tuning" | "experiment" | "debug" | "build"
    what: str


KNOBS: dict[str, Knob] = {
    # -- operation / deployment
    "SS_DEVICE": Knob("LOCAL_RANK", "framework/gpu.py", "ops",
                      "pin every rank to one device (multi-rank rehearsal on one GPU, gloo)"),
    "SS_BENCH_DEVICE": Knob("LOCAL_RANK", "bench.py", "ops", "same, for bench.py"),
    "SS_BENCH_TRACE_AFTER": Knob("unset", "bench.py", "ops",
                                 "dump every thread's Python stack to stderr after S seconds"),
    "SS_BENCH_ROUND_TIMEOUT": Knob("300", "bench.py", "ops",
                                   "seconds without a finished step before the bench aborts"),
    "SS_FAULT": Knob("", "parallel/watchdog.py", "ops",
                     "fault injection: hang|crash|slow:rank=R:step=S (once), "
                     "delay:<rank>:<ms> (a straggler: sleeps every step)"),
    "SS_LOG_LEVEL": Knob("WARNING", "utils/logging.py, csrc/host/common.h", "ops",
                         "log level (Python and the native runtime)"),
    "SS_LOCAL_IP": Knob("auto", "csrc/host/transfer.h", "ops",
                        "address the host-mode roles advertise"),
    "SS_CAL_PICK": Knob("", "models/base.py", "debug",
                        "sync|ahead: force the pull-ahead calibration's outcome (it still "
                        "measures both)"),
    "SS_GRAPH": Knob("1", "models/base.py", "ops",
                     "0: enable_graph() declines (replay is requested by config `graph` or "
                     "bench --graph); force: replay even with more than 4 ranks on one GPU "
                     "(declined by default: ~21 ms per round measured)"),
    # -- build
    "SS_OFFLOAD_ARCH": Knob("gfx950", "_build.py", "build", "HIP offload target"),
    "SS_NO_AUTOBUILD": Knob("0", "_native.py", "build",
                            "1: never build on import; a missing extension is an error"),
    # -- engine / table (defaults are the measured best)
    "SS_ENGINE_DEPTH": Knob("8 one GPU, 4 N>1", "parallel/engine.py", "tuning",
                            "route-buffer ring depth (>= 3 for pull-ahead; one GPU 8 vs 4: "
                            "0.791-0.797 vs 0.802-0.806 ms/step; 4 vs 3: 1.008 vs 1.018)"),
    "SS_PULL_AHEAD": Knob("auto", "parallel/engine.py", "tuning",
                          "pull rounds i+1..i+k while round i computes: auto = the models that "
                          "opt in (FM, word2vec), and at N>1 the bench / launcher calibration "
                          "times synchronous vs pulled-ahead steps on the live world and keeps "
                          "the faster; 1 = every model at N>1, 0 = none"),
    "SS_DEDUP": Knob("bucket", "ops/dedup.py", "tuning",
                     "bucket: LDS dedup per hash bucket; hash: global scratch table"),
    "SS_TABLE_G": Knob("auto", "ops/table.py", "tuning", "lanes per table row"),
    "SS_TABLE_LAYOUT": Knob("auto", "ops/table.py", "tuning",
                            "slot layout: rowfirst (width <= 2) / keyfirst"),
    "SS_TABLE_PREFILL": Knob("1", "ops/table.py", "tuning",
                             "zero-init tables pre-filled with the init row (insert = CAS only)"),
    "SS_TABLE_REGIONS": Knob("1", "ops/table.py", "tuning",
                             "scalar 16-byte LR slots: split the shard into 2^k probe regions "
                             "(>= 1024 slots each) so one dedup bucket owns its regions' inserts "
                             "(0: one region, every insert a device CAS)"),
    "SS_SERVER_STREAM": Knob("auto", "parallel/engine_dist.py", "tuning",
                             "N>1 over xGMI: the server half of each round (keys in, merge, "
                             "lookup, rows out; gradients in, merge + update) on its own "
                             "highest-priority stream; auto = when every rank has its own "
                             "device AND the bench / launcher calibration measures it within "
                             "1 % of the step without it (PipelinedWorker."
                             "calibrate_server_stream), 1 = always, 0 = on the main stream"),
    "SS_CAL_SERVER_STREAM": Knob("", "models/base.py", "debug",
                                 "0|1: force the server-stream calibration's outcome (it still "
                                 "measures both)"),
    "SS_MAIN_PRIO": Knob("0", "bench.py", "experiment",
                         "1: bench.py runs the step's main stream at the highest stream priority"),
    "SS_ROUTE_CUS": Knob("0", "parallel/engine.py", "experiment",
                         "n > 0: the route stream runs on n of the device's CUs (CU-masked "
                         "stream), leaving the rest to the main stream"),
    "SS_CLAIM_T": Knob("256", "csrc/hip/table.hip", "tuning",
                       "claimed pull: threads per bucket workgroup (256 / 512 / 1024: 0.795 / "
                       "0.833 / 0.843 ms per bench step on one box)"),
    "SS_SRV_FILL_FUSED": Knob("1", "csrc/hip/round_engine.cpp", "tuning",
                              "N>1 servers, claimed scalar pulls: the response fill (rows per "
                              "received position) fused into the pull (0: separate kernel)"),
    "SS_XCHG": Knob("auto", "bench.py, framework/gpu.py", "tuning",
                    "sparse LR N>1 xGMI rounds: unique = each source's unique keys, merged "
                    "on the worker first; records = every occurrence shipped, the servers "
                    "dedup and merge (less kernel work per rank at N <= 2, twice the link "
                    "bytes); auto (bench.py) = both timed on the live world after the "
                    "warm-up, the faster kept (the launcher runs unique)"),
    "SS_REC_GROUP": Knob("0", "parallel/engine.py", "tuning",
                         "1: N>1 record exchange with the unique layout's source buckets, each "
                         "bucket's records grouped by the servers' sub-bucket (measured slower "
                         "than the default 3584 / N records per source bucket at 2 and 4 ranks)"),
    "SS_BD_DBG": Knob("0", "csrc/hip/bdedup.hip", "debug",
                      "measurement only, wrong results: k_bd_reduce bits 1 = plain LDS stores, "
                      "2 = no gradient gather, 4 = no table stores, 8 = atomics for single keys"),
    "SS_XGMI_CACHED": Knob("0", "csrc/hip/xgmi.h", "experiment",
                           "1 (one-rank arenas only): the mailbox arenas as ordinary cached "
                           "memory — measures what the uncached mailbox costs its local readers"),
    "SS_CAL_XCHG": Knob("", "models/base.py", "debug",
                        "debug: force calibrate_exchange's outcome (unique / records)"),
    "SS_REC_OCC": Knob("own", "parallel/engine_dist.py", "tuning",
                       "record exchange: own = this rank's own records' rows go to a cached "
                       "buffer and their gradients are read by the server merge through spj "
                       "(never written per occurrence); arena = both through the mailbox, "
                       "like the peers' records"),
    "SS_SRV_STAGE": Knob("0", "parallel/engine_dist.py", "tuning",
                         "1: N>1 xGMI servers stream the peers' gradient rows out of the "
                         "uncached mailbox into a cached buffer before the merge gathers them "
                         "(measured neutral at 4 / 8 ranks on one GPU)"),
    "SS_W2V_FUSE": Knob("1", "models/word2vec.py", "tuning",
                        "one GPU: the word2vec occurrence-row reduce runs the optimizer update "
                        "of single-item keys itself; the apply kernel only the rest (0: reduce, "
                        "then apply every key)"),
    "SS_CLAIM": Knob("1", "parallel/engine.py", "tuning",
                     "one GPU, region tables, synchronous rounds: the pull claims new keys' "
                     "slots in LDS and the fused merge stores [w | h | key] (0: CAS inserts)"),
    "SS_BD_NCH": Knob("128", "csrc/hip/bdedup.hip", "tuning",
                      "max count/scatter chunks (1 GPU 512 -> 128: 0.93 -> 0.89 ms/step; "
                      "N>1 path 128 / 256 / 512: 1.06 / 1.03 / 1.05)"),
    "SS_BD_XCD": Knob("0", "csrc/hip/bdedup.hip", "tuning",
                      "1: scatter chunks in XCD-aware order (blocks b, b+8 share an XCD and get "
                      "adjacent chunks; measured neutral)"),
    "SS_BD_SKT": Knob("16", "csrc/hip/bdedup.hip", "tuning",
                      "sorted scatter: largest keys per thread per LDS tile (16 / 8 / 4 / 2; "
                      "halved for 12-byte records and when the bucket table needs the LDS)"),
    "SS_BD_SORT": Knob("1", "csrc/hip/bdedup.hip", "tuning",
                       "route scatter through an LDS counting sort per tile, stored in bucket "
                       "order (0: one random store per key)"),
    "SS_BD_CNT": Knob("1024", "csrc/hip/bdedup.hip", "tuning",
                      "count workgroup size"),
    "SS_BD_REC": Knob("auto", "csrc/hip/bdedup.hip", "tuning",
                      "key bytes of the scatter -> dedup hand-off (keys and pj as two arrays): "
                      "auto = 4 when every key of the call fits 32 bits, else 8; 8 fixed"),
    "SS_SLOT32": Knob("1", "swiftsnails_amd/parallel/engine.py", "tuning",
                      "one GPU, scalar (w, h) snapshot rows, shard under 2^31 slots: the pull "
                      "stores 4-byte slot indices for the fused merge + update (0: 8 bytes)"),
    "SS_SRV_AHEAD": Knob("1", "swiftsnails_amd/parallel/engine.py", "tuning",
                         "N>1 xGMI path, synchronous rounds: wait for the round's keys and "
                         "merge them into the server's distinct keys on the route stream, a "
                         "round ahead (0: at the head of the pull; pulled-ahead rounds always "
                         "keep them in the pull)"),
    "SS_PULL_VEC": Knob("1", "csrc/hip/table.hip", "tuning",
                        "wide fp32 rows (dim 32/64/128): pull and apply with 8 lanes per key "
                        "and 16-byte row vectors (0: one lane group per key)"),
    "SS_BD_TARGET": Knob("3584", "csrc/hip/bdedup.hip", "tuning",
                         "one rank: target occurrences per dedup bucket (1024..3584; 3584 / 3072 "
                         "/ 2048: 0.774-0.785 / 0.790 / 0.801-0.806 ms per bench step)"),
    "SS_BD_TARGET_DIST": Knob("3072", "csrc/hip/bdedup.hip, csrc/hip/server.hip", "tuning",
                              "N>1 unique-key layout: occurrences per source bucket (512..4096; "
                              "the servers' sub-bucket count follows)"),
    "SS_SRV_SUB": Knob("auto", "csrc/hip/server.hip", "tuning",
                       "N>1 servers: sub-buckets per bucket (auto: from the sources' bucket "
                       "size and count)"),
    "SS_BD_CS": Knob("1024", "csrc/hip/bdedup.hip", "tuning", "column-scan workgroup size"),
    "SS_BD_CT": Knob("1024", "csrc/hip/bdedup.hip", "tuning", "scatter workgroup size"),
    "SS_BD_RT": Knob("1024", "csrc/hip/bdedup.hip", "tuning", "reduce workgroup size"),
    "SS_CLAIM_TS": Knob("8192", "csrc/hip/table.hip", "tuning",
                        "claimed pull: LDS claim-set entries (8192, or 4096: 32 instead of "
                        "48 KB of LDS per workgroup)"),
    "SS_CLAIM_KR": Knob("1", "csrc/hip/table.hip", "tuning",
                        "claimed pull: keys per thread whose first probe loads are in flight "
                        "together (1 / 4 / 8; 4 and 8 measured slower)"),
    "SS_BD_ROCC": Knob("4", "csrc/hip/bdedup.hip", "tuning",
                       "k_bd_reduce: occurrences (and fused-update rows) per thread in flight, "
                       "2 or 4"),
    "SS_GEN_R": Knob("8", "csrc/hip/models.hip", "tuning",
                     "synthetic CTR generator: sample groups per workgroup (1 / 2 / 4 / 8)"),
    "SS_LR_FWD_R": Knob("4", "csrc/hip/segreduce.hip", "tuning",
                        "packed LR forward (one-gather mode): sample groups per workgroup, "
                        "their gathers in flight together (1 / 2 / 4 / 8; 8 measured 4 % slower)"),
    "SS_LR_FWD": Knob("auto", "csrc/hip/segreduce.hip", "tuning",
                      "LR forward layout: packed | group (auto by lane utilisation)"),
    "SS_FM_FUSE": Knob("0", "models/fm.py", "experiment",
                       "1: one GPU, FM's AdaGrad update fused into the sorted gradient merge "
                       "(rows as 8- + 16-byte vectors per thread; 0.570-0.573 vs 0.542-0.546 "
                       "ms/step for the merge + k_apply_st default)"),
    "SS_FM_REDUCE": Knob("sorted", "csrc/hip/bdedup.hip, models/fm.py", "tuning",
                         "FM gradient merge: sorted lists, or atomic (LDS float atomics)"),
    "SS_W2V_EARLY_SLOT": Knob("1", "csrc/hip/w2v.hip", "tuning",
                              "word2vec occurrence reduce with the fused update: load the key's "
                              "slot index beside the first gathers (1) or after them (0)"),
    "SS_W2V_PP_ITEMS": Knob("2", "csrc/hip/w2v.hip", "tuning",
                            "word2vec per-pair occurrence reduce: items per half-wave (2: two "
                            "independent item chains in lock step, 1: the one-item kernel)"),
    "SS_W2V_PP_QF": Knob("2", "csrc/hip/w2v.hip", "tuning",
                         "word2vec per-pair two-item reduce: occurrences per item and round "
                         "(2 or 4)"),
    "SS_W2V_PP_STAGES": Knob("3", "csrc/hip/w2v.hip", "tuning",
                             "word2vec per-pair negatives (K <= 5): pipeline stages of the "
                             "pair kernel (3 or 4); 2 = the any-K kernel"),
    "SS_W2V_MFMA": Knob("bf16", "models/word2vec.py", "tuning",
                        "word2vec tile: bf16 MFMA (77 KB LDS) or f32 (116 KB)"),
    "SS_RCCL_COMMS": Knob("1", "parallel/transport.py, bench.py", "ops",
                          "N>1 over RCCL: 1 = one communicator, every collective on one comm "
                          "stream in program order (conservative); 3 = data / count / pull "
                          "communicators on the engine's three streams"),
    "SS_XGMI_TIMEOUT": Knob("120", "parallel/xgmi.py", "ops",
                            "seconds a mailbox wait spins for a peer before it gives up (sticky "
                            "error raised at the next check point)"),
    "SS_XGMI_BPP": Knob("max(128, 1024 / world)", "parallel/xgmi.py", "tuning",
                        "workgroups per peer of a mailbox put"),
    "SS_XGMI_SELF": Knob("1", "csrc/hip/round_engine.cpp", "tuning",
                         "1: a rank's own segment of the keys / rows / gradients exchange is read "
                         "in place by its consumer instead of copied into its own arena by the "
                         "put (1/N of the put bytes; all of them at N = 1); 0: copied"),
    "SS_XGMI_LITMUS_TIMEOUT": Knob("30", "parallel/xgmi.py", "ops",
                                   "seconds a start-up litmus wait spins before the tier counts "
                                   "as failed (timeout: no further xGMI tier, RCCL)"),
    "SS_XGMI_VERIFY": Knob("0", "parallel/xgmi.py, csrc/hip/xgmi.hip", "ops",
                           "1: every put block writes a round tag after its payload, every "
                           "wait checks all tags (a flag that overtook its data raises at the "
                           "next round's poll)"),
    "SS_XGMI_FORCE_TIER": Knob("(none)", "parallel/xgmi.py", "ops",
                               "fenced: fail the drain tier's litmus on purpose; rccl: fail both "
                               "xGMI tiers (proves each step of the fallback chain)"),
    "SS_XGMI_FENCE_ALL": Knob("0", "parallel/xgmi.py", "ops",
                              "1: the fenced tier releases towards every peer, also peers on "
                              "the same device (tests of the tier with all ranks on one GPU)"),
    # -- experiments (measured slower or neutral; kept for re-measurement)
    "SS_ENGINE_GENERAL": Knob("0", "parallel/engine.py, bench.py", "experiment",
                              "run a 1-GPU job through the N>1 path (1: loopback, rccl: a size-1 "
                              "RCCL communicator, xgmi: a size-1 mailbox arena)"),
    "SS_STALENESS": Knob("1", "parallel/engine.py", "ops",
                         "pull-ahead depth and bound k (<= ring depth - 2): rounds i+1..i+k "
                         "are pulled while round i computes, each pull waits for the push k+1 "
                         "rounds back; 0: synchronous rounds; ring: one ahead, bounded by the "
                         "route-ring depth only (FM 0.655 -> 0.620 ms/step, word2vec 0.125 -> "
                         "0.118; N>1 LR path unchanged)"),
    "SS_PULL_STREAM": Knob("model (word2vec 1, FM 0)", "parallel/engine.py", "tuning",
                           "one GPU with pull-ahead: the pulled-ahead round's table lookup on "
                           "its own stream, beside the next round's dedup (word2vec 0.128 -> "
                           "0.125 ms/step; FM 0.655 -> 0.685, so off there)"),
    "SS_W2V_WIN_GRID": Knob("one per tile (atomic mode: CUs / 2)", "csrc/hip/w2v.hip", "tuning",
                            "grid of the windowed word2vec tile kernel (workgroups walk tiles; "
                            "0: one per tile); half the CUs leaves CUs to the route stream's "
                            "dedup when the tile is atomic-bound (0.143 -> 0.123 ms/step), one "
                            "per tile is faster with occurrence-row stores (0.101 -> 0.092)"),
    "SS_GRAPH_STEPS": Knob("4 x depth", "models/base.py", "tuning",
                           "steps per hipGraph: 1, or a multiple of the ring depth (word2vec "
                           "4 / 8 / 16 / 32: 0.093 / 0.088 / 0.086 / 0.084 ms/step)"),
    # -- debug
    "SS_BD_DEBUG": Knob("0", "ops/dedup.py", "debug",
                        "per-bucket dedup phase timestamps"),
}


def table() -> str:
    rows = ["| knob | default | kind | read in | what |", "|---|---|---|---|---|"]
    for k in sorted(KNOBS):
        v = KNOBS[k]
        rows.append(f"| `{k}` | {v.default} | {v.kind} | `{v.where}` | {v.what} |")
    return "\n".join(rows)


if __name__ == "__main__":  # pragma: no cover
    print(table())
