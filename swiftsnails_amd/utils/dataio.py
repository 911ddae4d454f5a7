"""File-backed training data with native parsing and asynchronous prefetch.

The reference apps read text data through ``scan_file_by_line`` /
``LineFileReader`` and the ``BaseAlgorithm::parse_record(line)`` hook
(/root/reference/src/utils/file.h:14-33, utils/string.h:89-114,
core/framework/SwiftWorker.h:19-30); the word2vec corpus format is the one
written by src/tools/gen-word2vec-data.py.  Here parsing and batch assembly
are native (``csrc/host/dataio.h``: memory-mapped file, per-thread line
ranges, GIL released) and Python only keeps a ring of pinned host buffers in
flight:

    fill (C++ threads) -> pinned host buffer -> async H2D copy on the caller's
    (route) stream -> event -> buffer reused ``prefetch`` steps later

Both sources are drop-in replacements for the synthetic generators
(``CtrSynth`` / ``W2VSynth``): same attributes the workers read and the same
``generate(step, rank, world, ...)`` call.  Rank ``r`` of a ``world``-rank job
reads its own 1/world of the file (data parallelism).

``FileCtrSource(resident="hbm")`` (the default on a GPU when the shard fits
in half of the free HBM) uploads the parsed shard (CSR: offsets, keys,
values, labels) to the GPU once and cuts each step's padded batch out of it
with one streaming kernel (``csrc/hip/data.hip``): no per-step host fill and
no per-step PCIe copy (82 MB for a 262144 x 39 batch), and the step becomes
hipGraph-capturable (the kernel can read its step from device memory).
``FileCorpusSource(resident="hbm")`` does the same for a word2vec corpus: the
tokens, sentence index, noise table and keep probabilities go to HBM and the
skip-gram sampler runs on the device, bit-identical to the host sampler.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Optional

import torch

from .._native import host

TILE = 64


class _PinnedRing:
    """Ring of pinned host buffer sets, each refilled by a native fill job once
    the H2D copy that last read it has completed."""

    def __init__(self, depth: int, shapes: Dict[str, tuple], pin: bool):
        self.depth = depth
        self.bufs = [{k: torch.empty(n, dtype=dt, pin_memory=pin) for k, (n, dt) in shapes.items()}
                     for _ in range(depth)]
        self.events = [None] * depth
        self.futures: Dict[int, object] = {}
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="ss-data")

    def submit(self, step: int, fill):
        if step in self.futures:
            return
        slot = step % self.depth
        ev = self.events[slot]

        def job():
            if ev is not None:
                ev.synchronize()  # the previous H2D copy out of this slot is done
            fill(step, self.bufs[slot])
            return slot

        self.events[slot] = None
        self.futures[step] = self.pool.submit(job)

    def take(self, step: int, fill):
        self.submit(step, fill)
        slot = self.futures.pop(step).result()
        for s in range(step + 1, step + self.depth):  # keep the other slots busy
            self.submit(s, fill)
        return slot, self.bufs[slot]

    def mark_copied(self, slot: int, stream):
        if torch.cuda.is_available() and stream is not None:
            ev = torch.cuda.Event()
            ev.record(stream)
            self.events[slot] = ev

    def close(self):
        self.pool.shutdown(wait=True)


def _ext_stream(stream):
    if stream is None or not torch.cuda.is_available():
        return None
    if isinstance(stream, int):
        return torch.cuda.ExternalStream(stream)
    return stream


OUT_BIT = 1 << 40  # word2vec output-embedding key bit (Corpus::kOutBit)


def _device(device) -> torch.device:
    return torch.device(device) if device is not None else torch.device(
        "cuda", torch.cuda.current_device())


def _choose_residency(resident, device, nbytes: int) -> str:
    """``hbm`` | ``host`` for a data source: ``auto``/None picks ``hbm`` on a
    GPU when the source's device copy fits in half of the free HBM."""
    if resident not in (None, "auto", "hbm", "host"):
        raise ValueError(f"data residency {resident!r}: hbm | host | auto")
    if resident in ("hbm", "host"):
        if resident == "hbm" and not torch.cuda.is_available():
            raise RuntimeError("data_resident: hbm needs a GPU")
        return resident
    if not torch.cuda.is_available():
        return "host"
    return "hbm" if nbytes <= torch.cuda.mem_get_info(_device(device))[0] // 2 else "host"


class FileCtrSource:
    """Sparse CTR batches from a libsvm (``label idx[:val] ...``) or categorical
    TSV (``label<TAB>tok<TAB>tok...``) file, padded to ``num_fields`` keys per
    sample (short rows padded with the EMPTY key, which the dedup skips)."""

    def __init__(self, path: str, fmt: str = "libsvm", batch_size: int = 65536,
                 num_fields: Optional[int] = None, rank: int = 0, world: int = 1,
                 nthreads: int = 8, prefetch: int = 3, pin: Optional[bool] = None,
                 resident: Optional[str] = None, device=None):
        self.ds = host().SparseDataset(path, fmt, nthreads, rank, world)
        if self.ds.rows == 0:
            raise ValueError(f"{path}: no rows for shard {rank}/{world}")
        self.batch_size = int(batch_size)
        self.num_fields = int(num_fields or self.ds.max_nnz)
        self.has_values = bool(self.ds.has_values)
        self.nthreads = nthreads
        # a synthetic-compatible attribute (table sizing when no capacity is set)
        self.num_features = max(1, self.ds.nnz)
        self.resident = _choose_residency(resident, device, self.device_bytes())
        self.ring = None
        if self.resident == "hbm":
            self._upload(device)
            return
        n = self.batch_size * self.num_fields
        shapes = {"keys": (n, torch.int64), "labels": (self.batch_size, torch.float32)}
        if self.has_values:
            shapes["vals"] = (n, torch.float32)
        pin = torch.cuda.is_available() if pin is None else pin
        self.ring = _PinnedRing(max(1, prefetch), shapes, pin)

    def device_bytes(self) -> int:
        """HBM the resident copy of this shard takes."""
        ds = self.ds
        return 8 * (ds.rows + 1) + 8 * ds.nnz + 4 * ds.rows + (4 * ds.nnz if self.has_values else 0)

    def _upload(self, device):
        import numpy as np

        dev = _device(device)
        ds = self.ds
        self.device = dev
        self.d_offs = torch.from_numpy(np.asarray(ds.offsets()).view(np.int64)).to(dev)
        self.d_keys = torch.from_numpy(np.asarray(ds.keys()).view(np.int64)).to(dev)
        self.d_labels = torch.from_numpy(np.asarray(ds.labels())).to(dev)
        self.d_vals = (torch.from_numpy(np.asarray(ds.vals())).to(dev) if self.has_values
                       else None)
        torch.cuda.synchronize(dev)

    @property
    def graph_capturable(self) -> bool:
        """Resident batches read their step from device memory in a replay."""
        return self.resident == "hbm"

    @property
    def rows(self) -> int:
        return self.ds.rows

    def steps_per_pass(self) -> int:
        """Steps of one pass over this rank's shard: every row once; the last
        batch of a pass wraps into the shard's start (no partial batches)."""
        return -(-self.ds.rows // self.batch_size)

    def _fill(self, step: int, buf):
        cursor = (step * self.batch_size) % self.ds.rows
        self.ds.fill(cursor, self.batch_size, self.num_fields, buf["keys"].data_ptr(),
                     buf["vals"].data_ptr() if "vals" in buf else 0, buf["labels"].data_ptr(),
                     self.nthreads)

    def generate(self, step: int, rank: int, world: int, keys: torch.Tensor,
                 labels: torch.Tensor, stream=None, xval: Optional[torch.Tensor] = None,
                 step_dev: int = 0, step_delta: int = 0):
        """Batch of ``step`` (rows [step*B, step*B + B) of this rank's shard,
        wrapping).  Resident: with ``step_dev`` (a device int64 pointer,
        hipGraph replays) the step is ``*step_dev + step_delta``."""
        if self.resident == "hbm":
            from .._native import hip

            st = stream if stream is not None else torch.cuda.current_stream()
            st = st.cuda_stream if hasattr(st, "cuda_stream") else int(st)
            B, F = self.batch_size, self.num_fields
            if keys.numel() < B * F or labels.numel() < B:
                raise ValueError("generate: output buffers smaller than the batch")
            for t in (keys, labels, xval):
                if t is not None and t.device != self.device:
                    raise ValueError(f"generate: HBM-resident batches are written on "
                                     f"{self.device}, got a buffer on {t.device}")
            hip().csr_batch(self.d_offs.data_ptr(), self.d_keys.data_ptr(),
                            self.d_vals.data_ptr() if self.d_vals is not None else 0,
                            self.d_labels.data_ptr(), self.ds.rows,
                            (step * B) % self.ds.rows, B, F, step_dev, step_delta,
                            keys.data_ptr(), xval.data_ptr() if xval is not None else 0,
                            labels.data_ptr(), st)
            return
        if step_dev:
            raise RuntimeError("host-resident file batches cannot be replayed from a graph")
        slot, buf = self.ring.take(step, self._fill)
        st = _ext_stream(stream)
        ctx = torch.cuda.stream(st) if st is not None else _null()
        with ctx:
            nb = keys.is_cuda
            keys.copy_(buf["keys"], non_blocking=nb)
            labels.copy_(buf["labels"], non_blocking=nb)
            if xval is not None:
                if "vals" in buf:
                    xval.copy_(buf["vals"], non_blocking=nb)
                else:
                    xval.fill_(1.0)
        self.ring.mark_copied(slot, st if st is not None else (
            torch.cuda.current_stream() if keys.is_cuda else None))

    def close(self):
        if self.ring is not None:
            self.ring.close()


from ..models.word2vec import W2VLayout  # noqa: E402  (key layouts shared with W2VSynth)


class FileCorpusSource(W2VLayout):
    """Skip-gram batches from a text corpus (one sentence per line; integer
    tokens are word ids, other tokens are hashed) in the ``W2VSynth`` key
    layouts: ``mode="window"`` (default) walks the rank's corpus shard in
    order, one run of B + 2W positions per step (every token is a center once
    per epoch, its contexts are its sentence neighbours within a reduced
    window); ``mode="pairs"`` samples i.i.d. centers and 2W contexts each."""

    def __init__(self, path: str, batch_size: int = 16384, window: int = 5, negatives: int = 5,
                 rank: int = 0, world: int = 1, min_count: int = 1, sample: float = 0.0,
                 seed: int = 1234, nthreads: int = 8, prefetch: int = 3,
                 pin: Optional[bool] = None, resident: Optional[str] = None, device=None,
                 mode: str = "window", neg_mode: str = "shared"):
        self.corpus = host().Corpus(path, nthreads, rank, world, min_count, sample)
        self.batch_size = int(batch_size)
        self.window = int(window)
        self.negatives = int(negatives)
        self.mode = mode
        self.neg_mode = neg_mode
        self._check_mode()
        self.seed = int(seed) + 7919 * rank
        self.nthreads = nthreads
        self.vocab = max(1, self.corpus.vocab_size)
        self.ring = None
        self.resident = _choose_residency(resident, device, self.device_bytes())
        if self.resident == "hbm":
            self._upload(device)
            return
        pin = torch.cuda.is_available() if pin is None else pin
        bufs = {"keys": (self.n_keys, torch.int64)}
        if self.mode == "window":
            bufs["meta"] = (self.run_len, torch.int32)
        self.ring = _PinnedRing(max(1, prefetch), bufs, pin)

    def device_bytes(self) -> int:
        """HBM the resident sampler state takes (tokens, sentence index, noise
        table, keep probabilities)."""
        c = self.corpus
        n = c.size
        return 8 * n + 4 * n + 8 * (c.sentences + 1) + 8 * (1 << 22) + (4 * n if c.subsampled else 0)

    def _upload(self, device):
        import numpy as np

        dev = _device(device)
        c = self.corpus
        self.device = dev
        self.d_tokens = torch.from_numpy(np.asarray(c.tokens()).view(np.int64)).to(dev)
        self.d_soffs = torch.from_numpy(np.asarray(c.sent_offsets()).view(np.int64)).to(dev)
        self.d_sof = torch.from_numpy(np.asarray(c.sent_of()).view(np.int32)).to(dev)
        self.d_table = torch.from_numpy(np.asarray(c.noise_table()).view(np.int64)).to(dev)
        self.d_keep = (torch.from_numpy(np.asarray(c.keep_per_token())).to(dev)
                       if c.subsampled else None)
        torch.cuda.synchronize(dev)

    @property
    def graph_capturable(self) -> bool:
        return self.resident == "hbm"

    def steps_per_pass(self) -> int:
        """Steps of one pass over this rank's corpus shard: window mode walks
        every token as a center once per pass; pairs mode draws as many
        centers."""
        return -(-self.corpus.size // self.batch_size)

    def _fill(self, step: int, buf):
        if self.mode == "window":
            self.corpus.fill_skipgram_window(self.seed, step, self.batch_size, self.window,
                                             self.n_neg, buf["keys"].data_ptr(),
                                             buf["meta"].data_ptr())
            return
        self.corpus.fill_skipgram(self.seed, step, self.batch_size, self.contexts, self.window,
                                  self.n_neg, buf["keys"].data_ptr(), self.nthreads)

    def generate(self, step: int, rank: int, world: int, keys: torch.Tensor, stream=None,
                 step_dev: int = 0, step_delta: int = 0, meta: Optional[torch.Tensor] = None):
        if self.mode == "window" and (meta is None or meta.numel() < self.run_len):
            raise ValueError("window mode: generate() needs a meta buffer of run_len int32")
        if self.resident == "hbm":
            from .._native import hip

            if keys.device != self.device or keys.numel() < self.n_keys:
                raise ValueError("generate: the key buffer must hold n_keys on the corpus' device")
            st = stream if stream is not None else torch.cuda.current_stream()
            st = st.cuda_stream if hasattr(st, "cuda_stream") else int(st)
            if self.mode == "window":
                if meta.device != self.device:
                    raise ValueError("generate: the meta buffer must be on the corpus' device")
                hip().w2v_corpus_window(self.d_tokens.data_ptr(), self.d_sof.data_ptr(),
                                        self.corpus.sentences, self.d_table.data_ptr(),
                                        self.d_table.numel(),
                                        self.d_keep.data_ptr() if self.d_keep is not None else 0,
                                        self.d_tokens.numel(), self.seed, step, step_dev,
                                        step_delta, self.batch_size, self.window,
                                        self.n_neg, OUT_BIT, keys.data_ptr(),
                                        meta.data_ptr(), st)
                return
            hip().w2v_corpus_batch(self.d_tokens.data_ptr(), self.d_soffs.data_ptr(),
                                   self.d_sof.data_ptr(), self.d_table.data_ptr(),
                                   self.d_table.numel(),
                                   self.d_keep.data_ptr() if self.d_keep is not None else 0,
                                   self.d_tokens.numel(), self.seed, step, step_dev, step_delta,
                                   self.batch_size, self.contexts, self.window,
                                   self.n_neg, OUT_BIT, keys.data_ptr(), st)
            return
        if step_dev:
            raise RuntimeError("host-fed corpus batches cannot be replayed from a graph")
        slot, buf = self.ring.take(step, self._fill)
        st = _ext_stream(stream)
        ctx = torch.cuda.stream(st) if st is not None else _null()
        with ctx:
            keys.copy_(buf["keys"], non_blocking=keys.is_cuda)
            if self.mode == "window":
                meta.copy_(buf["meta"], non_blocking=meta.is_cuda)
        self.ring.mark_copied(slot, st if st is not None else (
            torch.cuda.current_stream() if keys.is_cuda else None))

    def close(self):
        if self.ring is not None:
            self.ring.close()


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def rank_data_path(path: str, rank: int, world: int) -> tuple[str, int, int]:
    """(file, shard, nshards) a rank reads: ``data_path`` with ``{rank}`` in
    it names one file per rank (the reference's per-worker input split,
    /root/reference/src/tools/run_worker.sh:4,13 — each worker trains on
    its own data file), read whole; otherwise the rank takes the rank-th
    contiguous 1/world of one shared file."""
    if "{rank}" in path:
        return path.replace("{rank}", str(rank)), 0, 1
    return path, rank, world


def make_ctr_source(cfg, rank: int = 0, world: int = 1, device=None):
    """Config keys: data_path, data_format (libsvm|ctr), batch_size, num_fields,
    data_resident (auto|hbm|host)."""
    path, rank, world = rank_data_path(cfg.get("data_path"), rank, world)
    return FileCtrSource(path, cfg.get("data_format", "libsvm"),
                         batch_size=int(cfg.get("batch_size", 65536)),
                         num_fields=int(cfg.get("num_fields", 0) or 0) or None,
                         rank=rank, world=world,
                         nthreads=int(cfg.get("data_threads", 8)),
                         resident=cfg.get("data_resident", "auto"), device=device)


def make_corpus_source(cfg, rank: int = 0, world: int = 1, device=None):
    """Config keys: data_path, batch_size, window, negatives, min_count, sample,
    data_resident (auto|hbm|host), w2v_mode (window|pairs), neg_mode (shared|per_pair)."""
    path, shard, nshards = rank_data_path(cfg.get("data_path"), rank, world)
    return FileCorpusSource(path, batch_size=int(cfg.get("batch_size", 16384)),
                            seed=1234 + 7919 * (rank - shard),  # negatives differ per rank
                            window=int(cfg.get("window", 5)),
                            negatives=int(cfg.get("negatives", 5)), rank=shard, world=nshards,
                            min_count=int(cfg.get("min_count", 1)),
                            sample=float(cfg.get("sample", 0.0)),
                            nthreads=int(cfg.get("data_threads", 8)),
                            resident=cfg.get("data_resident", "auto"), device=device,
                            mode=cfg.get("w2v_mode", "window"),
                            neg_mode=cfg.get("neg_mode", "shared"))
