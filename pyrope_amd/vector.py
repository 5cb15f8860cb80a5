"""Host-side mirror of the reference plugin surface for the scan path.

Restates the C# contract `IVectorIndex` (reference
src/Pyrope.GarnetServer/Vector/IVectorIndex.cs:5-31), `SearchOptions`
(SearchOptions.cs:3), `ICentroidsProvider` (ICentroidsProvider.cs:14), the
`DeltaVectorIndex` composite (DeltaVectorIndex.cs) and the registry factory
branch (Services/VectorIndexRegistry.cs:81-113) over the C ABI of
libpyrope_hip.so.  This is what the C# P/Invoke shim does:
string ids <-> int64 labels, argument validation with the reference's
exception types and messages, one call per batch.
"""
from __future__ import annotations

import ctypes as C
import enum
import json
import warnings
import os
import re
import threading
from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (ArgumentException, ArgumentNullException, ArgumentOutOfRangeException, FormatException,
                   InvalidOperationException, check, ptr)


class VectorMetric(enum.IntEnum):  # IVectorIndex.cs:5-10
    L2 = 0
    InnerProduct = 1
    Cosine = 2


@dataclass(frozen=True)
class SearchResult:  # IVectorIndex.cs:12
    id: str
    score: float


@dataclass(frozen=True)
class IndexStats:  # IVectorIndex.cs:31
    count: int
    dimension: int
    metric: str


@dataclass(frozen=True)
class SearchOptions:  # SearchOptions.cs:3
    max_scans: Optional[int] = None
    nprobe: Optional[int] = None
    ef_search: Optional[int] = None


class IVectorIndex(ABC):  # IVectorIndex.cs:14-29
    dimension: int
    metric: VectorMetric

    @abstractmethod
    def add(self, id: str, vector: Sequence[float]) -> None: ...

    @abstractmethod
    def upsert(self, id: str, vector: Sequence[float]) -> None: ...

    @abstractmethod
    def delete(self, id: str) -> bool: ...

    @abstractmethod
    def search(self, query: Sequence[float], top_k: int,
               options: Optional[SearchOptions] = None) -> List[SearchResult]: ...

    @abstractmethod
    def build(self) -> None: ...

    @abstractmethod
    def snapshot(self, path: str) -> None: ...

    @abstractmethod
    def load(self, path: str) -> None: ...

    @abstractmethod
    def get_stats(self) -> IndexStats: ...


class ICentroidsProvider(ABC):  # ICentroidsProvider.cs:14
    @abstractmethod
    def get_centroids(self) -> Optional[List[np.ndarray]]: ...


def _validate_id(id: str) -> None:  # BruteForceVectorIndex.cs:386-389
    if id is None or str(id).strip() == "":
        raise ArgumentException("Id cannot be empty.")


class HipVectorIndex(IVectorIndex):
    """An IVectorIndex backed by libpyrope_hip.so (the C# shim's behaviour)."""

    KIND = _lib.PYR_FLAT

    def __init__(self, dimension: int, metric: VectorMetric, *, nlist: int = 100, m: int = 4, k: int = 256,
                 device: int = 0, default_nprobe: int = 0, device_mask: int = 0, shards: int = 0):
        """device_mask / shards: the multi-GPU index (IVF_FLAT; pyr_index_desc in include/pyrope_ann.h)."""
        if dimension <= 0:
            raise ArgumentOutOfRangeException("Dimension must be positive.")
        self.dimension = int(dimension)
        self.metric = VectorMetric(metric)
        self._L = _lib.load()
        desc = _lib.IndexDesc(self.KIND, self.dimension, int(self.metric), nlist, m, k, device, default_nprobe,
                              int(device_mask), int(shards), 0)
        h = C.c_void_p()
        check(self._L.pyr_index_create(C.byref(desc), C.byref(h)))
        self._h = h
        self._label_of: Dict[str, int] = {}
        self._id_of: Dict[int, str] = {}
        self._next_label = 0  # labels are never reused: above every label handed out so far

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.pyr_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- id <-> label (the shim's job) ----
    def _label(self, id: str) -> int:
        lab = self._label_of.get(id)
        if lab is None:
            lab = self._next_label
            self._next_label += 1
            self._label_of[id] = lab
            self._id_of[lab] = id
        return lab

    def _register_labels(self, labels: np.ndarray) -> None:
        """Caller-chosen labels (id = str(label)); later new ids get labels above all of them."""
        for lab in labels.tolist():
            self._label_of[str(lab)] = lab
            self._id_of[lab] = str(lab)
        if len(labels):
            self._next_label = max(self._next_label, int(labels.max()) + 1)

    def _vec(self, vector) -> np.ndarray:
        if vector is None:
            raise ArgumentNullException("vector")
        v = np.ascontiguousarray(vector, dtype=np.float32).reshape(-1)
        if v.size != self.dimension:
            raise ArgumentException("Vector dimension mismatch.")
        return v

    def _write(self, fn, ids: Sequence[str], x: np.ndarray) -> None:
        labels = np.array([self._label(i) for i in ids], dtype=np.int64)
        x = np.ascontiguousarray(x, dtype=np.float32).reshape(len(labels), self.dimension)
        check(fn(self._h, ptr(x, C.c_float), len(labels), ptr(labels, C.c_int64)))

    # ---- IVectorIndex ----
    def add(self, id: str, vector) -> None:
        _validate_id(id)
        self._write(self._L.pyr_index_add, [id], self._vec(vector))

    def upsert(self, id: str, vector) -> None:
        _validate_id(id)
        self._write(self._L.pyr_index_upsert, [id], self._vec(vector))

    def add_batch(self, ids: Sequence[str], x: np.ndarray) -> None:
        self._write(self._L.pyr_index_add, ids, x)

    def upsert_batch(self, ids: Sequence[str], x: np.ndarray) -> None:
        """Upsert of many rows in one call, applied in order (a repeated id: the last row wins)."""
        self._write(self._L.pyr_index_upsert, ids, x)

    def add_labels(self, labels: np.ndarray, x: np.ndarray, track_ids: bool = True) -> None:
        """Bulk add with caller-chosen int64 labels (id = str(label)).  track_ids=False skips the
        host id map (bulk loads that only ever read labels back, e.g. bench.py at 10^7+ rows)."""
        labels = np.ascontiguousarray(labels, dtype=np.int64)
        if track_ids:
            self._register_labels(labels)
        elif len(labels):
            self._next_label = max(self._next_label, int(labels.max()) + 1)
        x = np.ascontiguousarray(x, dtype=np.float32)
        check(self._L.pyr_index_add(self._h, ptr(x, C.c_float), len(labels), ptr(labels, C.c_int64)))

    def delete(self, id: str) -> bool:
        _validate_id(id)
        lab = self._label_of.get(id)
        if lab is None:
            return False
        labels = np.array([lab], np.int64)
        removed = np.zeros(1, np.uint8)
        check(self._L.pyr_index_remove(self._h, ptr(labels, C.c_int64), 1, ptr(removed, C.c_uint8)))
        return bool(removed[0])

    def build(self) -> None:
        check(self._L.pyr_index_build(self._h))

    def _params(self, options: Optional[SearchOptions]) -> _lib.SearchParams:
        p = _lib.SearchParams(-1, 0, -1)
        if options is not None:
            if options.nprobe is not None:
                p.nprobe = max(int(options.nprobe), 0)
            if options.max_scans is not None:
                p.max_scans = max(int(options.max_scans), 0)
        return p

    def search_batch(self, queries: np.ndarray, top_k: int, options: Optional[SearchOptions] = None):
        """Batched Search: returns (scores [nq,k] fp32, labels [nq,k] int64, counts [nq])."""
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dimension)
        nq = q.shape[0]
        kk = max(int(top_k), 0)
        s = np.empty((nq, kk), np.float32)
        lab = np.empty((nq, kk), np.int64)
        cnt = np.empty(nq, np.int32)
        p = self._params(options)
        check(self._L.pyr_index_search(self._h, ptr(q, C.c_float), nq, int(top_k), C.byref(p), ptr(s, C.c_float),
                                       ptr(lab, C.c_int64), ptr(cnt, C.c_int32)))
        return s, lab, cnt

    def search(self, query, top_k: int, options: Optional[SearchOptions] = None) -> List[SearchResult]:
        q = self._vec(query)
        s, lab, cnt = self.search_batch(q[None, :], top_k, options)
        return [SearchResult(self._id_of.get(int(lab[0, j]), str(int(lab[0, j]))), float(s[0, j]))
                for j in range(int(cnt[0]))]

    def set_coalescing(self, max_batch: int, max_wait_us: int) -> None:
        """Merge concurrent searches into device batches (pyr_index_set_coalescing); 0 turns it off."""
        check(self._L.pyr_index_set_coalescing(self._h, int(max_batch), int(max_wait_us)))

    def search_device(self, d_q: int, nq: int, top_k: int, d_scores: int, d_labels: int, d_counts: int = 0,
                      stream: int = 0, options: Optional[SearchOptions] = None, d_probes: int = 0,
                      nprobe: int = 0) -> None:
        """Search on device-resident buffers (raw device pointers, e.g. torch tensor.data_ptr()).
        d_probes / nprobe: caller-ranked probe lists (pyr_index_search_probed_device)."""
        p = self._params(options)
        if d_probes:
            check(self._L.pyr_index_search_probed_device(self._h, C.c_void_p(d_q), nq, int(top_k), C.byref(p),
                                                         C.c_void_p(d_probes), int(nprobe), C.c_void_p(d_scores),
                                                         C.c_void_p(d_labels), C.c_void_p(d_counts or None),
                                                         C.c_void_p(stream or None)))
            return
        check(self._L.pyr_index_search_device(self._h, C.c_void_p(d_q), nq, int(top_k), C.byref(p),
                                              C.c_void_p(d_scores), C.c_void_p(d_labels),
                                              C.c_void_p(d_counts or None), C.c_void_p(stream or None)))

    def probe_device(self, d_q: int, nq: int, d_probes: int, stream: int = 0,
                     options: Optional[SearchOptions] = None) -> int:
        """Coarse ranking only (pyr_index_probe_device): probe lists [nq][P] at d_probes; returns P."""
        p = self._params(options)
        out = C.c_int32()
        check(self._L.pyr_index_probe_device(self._h, C.c_void_p(d_q), nq, int(p.nprobe), C.c_void_p(d_probes),
                                             C.byref(out), C.c_void_p(stream or None)))
        return out.value

    # ---- list-sharded multi-GPU search (IVF_FLAT; pyrope_amd/dist.py ListShardedIvf) ----
    def set_list_samples(self, rows: np.ndarray, counts: np.ndarray, list_len: np.ndarray) -> None:
        """The replicated sample of every list: its first counts[l] <= 512 rows (in list order,
        concatenated) and list_len[l], its full length on the rank that owns it."""
        rows = np.ascontiguousarray(rows, dtype=np.float32).reshape(-1, self.dimension)
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        list_len = np.ascontiguousarray(list_len, dtype=np.int64)
        if counts.sum() != rows.shape[0] or len(list_len) != len(counts):
            raise ArgumentException("sample rows do not match their counts")
        check(self._L.pyr_index_set_list_samples(self._h, ptr(rows, C.c_float), ptr(counts, C.c_int64),
                                                 ptr(list_len, C.c_int64), len(counts)))

    def shard_prepare_device(self, d_q: int, nq: int, top_k: int, d_plan: int, stream: int = 0,
                             options: Optional[SearchOptions] = None) -> int:
        """Home rank: coarse ranking + T_q -> plan [nq][P + 1] at d_plan (with options.max_scans: [nq][2P + 1],
        the MaxScans budget left at each probe after T_q; shard_plan_stride); returns P."""
        p = self._params(options)
        out = C.c_int32()
        check(self._L.pyr_index_shard_prepare_device(self._h, C.c_void_p(d_q), nq, int(top_k), C.byref(p),
                                                     C.c_void_p(d_plan), C.byref(out), C.c_void_p(stream or None)))
        return out.value

    def shard_search_device(self, d_q: int, nq: int, top_k: int, d_plan: int, width: int, d_records: int,
                            stream: int = 0, budgets: bool = False) -> None:
        """Every rank: its owned lists against the gathered plans -> one record per query (budgets: the plans
        carry MaxScans budgets)."""
        check(self._L.pyr_index_shard_search_device(self._h, C.c_void_p(d_q), nq, int(top_k), C.c_void_p(d_plan),
                                                    int(width), int(bool(budgets)), C.c_void_p(d_records),
                                                    C.c_void_p(stream or None)))

    def shard_rerun_device(self, d_q: int, nq: int, top_k: int, d_plan: int, width: int, d_fails: int, nranks: int,
                           fcap: int, nq_home: int, d_records: int, stream: int = 0, budgets: bool = False) -> None:
        """Every rank: exact answers to the gathered failures [nranks][1 + fcap] -> records [nranks * fcap]."""
        check(self._L.pyr_index_shard_rerun_device(self._h, C.c_void_p(d_q), nq, int(top_k), C.c_void_p(d_plan),
                                                   int(width), int(bool(budgets)), C.c_void_p(d_fails), int(nranks),
                                                   int(fcap), int(nq_home), C.c_void_p(d_records),
                                                   C.c_void_p(stream or None)))

    def shard_info(self) -> dict:
        """The multi-GPU index's shards and its list-sharded step's counters (pyr_index_shard_info)."""
        a, b = C.c_int32(), C.c_int32()
        c, d, e, f = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        check(self._L.pyr_index_shard_info(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d), C.byref(e),
                                           C.byref(f)))
        return {"shards": a.value, "xport": {0: None, 1: "copy", 2: "rccl"}[b.value], "sharded_searches": c.value,
                "staged_searches": d.value, "last_max_failures": e.value, "last_extra_rounds": f.value}

    def set_centroids(self, centroids: np.ndarray) -> None:
        """Supply the coarse quantizer used by the next build() (pyr_index_set_centroids)."""
        c = np.ascontiguousarray(centroids, dtype=np.float32).reshape(-1, self.dimension)
        check(self._L.pyr_index_set_centroids(self._h, ptr(c, C.c_float), c.shape[0]))

    def reserve(self, rows: int) -> None:
        """Capacity hint for a bulk load of `rows` more rows (pyr_index_reserve); results unchanged."""
        check(self._L.pyr_index_reserve(self._h, int(rows)))

    def get_stats(self) -> IndexStats:
        cnt = C.c_int64()
        check(self._L.pyr_index_stats(self._h, C.byref(cnt), None, None))
        return IndexStats(int(cnt.value), self.dimension, self.metric.name)

    # ---- IVectorIndex.Snapshot / Load (IVectorIndex.cs:26-27) ----
    def snapshot(self, path: str) -> None:
        """The library's binary image at `path` (pyr_index_snapshot) plus the shim's id <-> label map
        at path + ".ids" (JSON), each written through a temp file and a rename.  The map records the
        image's nonce (16 random bytes every snapshot draws, pyr_image_nonce), so a crash between the
        two renames cannot pair a new image with the previous snapshot's map: load()
        then warns, ignores the stale map and falls back to str(label) ids."""
        if path is None or str(path).strip() == "":
            raise ArgumentException("Path cannot be empty.")
        check(self._L.pyr_index_snapshot(self._h, os.fsencode(str(path))))
        ids = {"next": self._next_label, "image_nonce": self._image_nonce(path),
               "ids": [[i, lab] for i, lab in self._label_of.items()]}
        tmp = str(path) + ".ids.tmp"
        with open(tmp, "w") as f:
            json.dump(ids, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, str(path) + ".ids")

    def _image_nonce(self, path) -> str:
        nonce = np.zeros(16, np.uint8)
        check(self._L.pyr_image_nonce(os.fsencode(str(path)), ptr(nonce, C.c_uint8)))
        return nonce.tobytes().hex()

    def load(self, path: str) -> None:
        if path is None or str(path).strip() == "":
            raise ArgumentException("Path cannot be empty.")
        check(self._L.pyr_index_load(self._h, os.fsencode(str(path))))
        self._label_of, self._id_of = {}, {}
        self._next_label = 0
        ids = None
        try:
            with open(str(path) + ".ids") as f:
                ids = json.load(f)
        except FileNotFoundError:
            pass
        if ids is not None and not self._map_matches(path, ids):
            warnings.warn(f"{path}.ids belongs to another image (nonce mismatch); ids fall back to "
                          "str(label)", RuntimeWarning, stacklevel=2)
            ids = None
        if ids is None:
            # an image without (its own) shim map, e.g. written by pyr_index_snapshot directly or by
            # another client: every loaded row's id is str(label), new ids get labels above them all
            self._register_labels(self.loaded_labels())
            return
        for i, lab in ids["ids"]:
            self._label_of[i] = lab
            self._id_of[lab] = i
        self._next_label = int(ids.get("next", 0))

    def _map_matches(self, path, ids) -> bool:
        """An id map pairs with the image whose nonce it recorded.  A map written before images carried a
        nonce (no 'image_nonce'; round 3's 'image': [size, mtime_ns]) pairs only with a nonce-less image
        (its nonce reads as zeros) whose size and mtime it recorded."""
        nonce = self._image_nonce(path)
        if "image_nonce" in ids:
            return ids["image_nonce"] == nonce
        if nonce != "00" * 16:
            return False
        img = ids.get("image")
        if img is None:
            return True
        st = os.stat(str(path))
        return [int(st.st_size), int(st.st_mtime_ns)] == [int(v) for v in img]

    def loaded_labels(self) -> np.ndarray:
        """Labels of every row the index holds (pyr_index_labels)."""
        n = C.c_int64(0)
        check(self._L.pyr_index_labels(self._h, None, C.byref(n)))
        out = np.zeros(max(n.value, 1), np.int64)
        n2 = C.c_int64(len(out))
        check(self._L.pyr_index_labels(self._h, ptr(out, C.c_int64), C.byref(n2)))
        return np.unique(out[: n2.value])

    # ---- introspection used by parity tests and the CPU baseline ----
    def ivf_layout(self):
        total = C.c_int64()
        nl = C.c_int32()
        check(self._L.pyr_index_get_centroids(self._h, None, C.byref(nl)))
        check(self._L.pyr_index_ivf_layout(self._h, None, None, None, C.byref(total)))
        off = np.zeros(nl.value + 1, np.int64)
        labels = np.zeros(total.value, np.int64)
        live = np.zeros(total.value, np.uint8)
        check(self._L.pyr_index_ivf_layout(self._h, ptr(off, C.c_int64), ptr(labels, C.c_int64),
                                           ptr(live, C.c_uint8), C.byref(total)))
        return off, labels, live

    def centroids_array(self) -> Optional[np.ndarray]:
        nl = C.c_int32()
        check(self._L.pyr_index_get_centroids(self._h, None, C.byref(nl)))
        if nl.value == 0:
            return None
        out = np.zeros((nl.value, self.dimension), np.float32)
        check(self._L.pyr_index_get_centroids(self._h, ptr(out, C.c_float), C.byref(nl)))
        return out


class BruteForceVectorIndex(HipVectorIndex):
    """FLAT (BruteForceVectorIndex.cs) -- the Delta head."""
    KIND = _lib.PYR_FLAT

    def __init__(self, dimension: int, metric: VectorMetric, **kw):
        super().__init__(dimension, metric, **kw)

    def search(self, query, top_k: int, options: Optional[SearchOptions] = None) -> List[SearchResult]:
        self._vec(query)
        if top_k <= 0:  # :278
            raise ArgumentOutOfRangeException("topK must be positive.")
        return super().search(query, top_k, options)

    @property
    def enable_quantization(self) -> bool:  # EnableQuantization (:25-40)
        return getattr(self, "_quant", False)

    @enable_quantization.setter
    def enable_quantization(self, value: bool) -> None:
        check(self._L.pyr_index_set_quantization(self._h, 1 if value else 0))
        self._quant = bool(value)

    def scan(self):  # :250-273 (compaction source): live rows in slot order
        """[(id, vector)] of the live rows in slot order (pyr_index_scan)."""
        n = C.c_int64()
        check(self._L.pyr_index_scan(self._h, None, None, C.byref(n)))
        labels = np.zeros(n.value, np.int64)
        x = np.zeros((n.value, self.dimension), np.float32)
        check(self._L.pyr_index_scan(self._h, ptr(labels, C.c_int64), ptr(x, C.c_float), C.byref(n)))
        return [(self._id_of.get(int(lab), str(int(lab))), x[i]) for i, lab in enumerate(labels.tolist())]

    def delete_many(self, ids: Sequence[str]) -> None:
        labels = np.array([self._label_of[i] for i in ids if i in self._label_of], np.int64)
        if len(labels):
            check(self._L.pyr_index_remove(self._h, ptr(labels, C.c_int64), len(labels), None))


class IvfFlatVectorIndex(HipVectorIndex, ICentroidsProvider):
    """IVF_FLAT (IvfFlatVectorIndex.cs)."""
    KIND = _lib.PYR_IVF_FLAT

    def __init__(self, dimension: int, metric: VectorMetric, n_list: int = 100, **kw):
        super().__init__(dimension, metric, nlist=n_list, **kw)
        self.n_list = n_list
        self.combine_nprobe = 3  # CombineNProbe (:14)

    def _params(self, options):
        p = super()._params(options)
        if options is None or options.nprobe is None:
            p.nprobe = max(int(self.combine_nprobe), 0)
        return p

    def get_centroids(self):  # :314-325
        c = self.centroids_array()
        return None if c is None else [row.copy() for row in c]


class IvfPqVectorIndex(HipVectorIndex):
    """IVF_PQ (IvfPqVectorIndex.cs + ProductQuantizer.cs)."""
    KIND = _lib.PYR_IVF_PQ

    def __init__(self, dimension: int, metric: VectorMetric, m: int, k: int, n_list: int, **kw):
        super().__init__(dimension, metric, nlist=n_list, m=m, k=k, **kw)
        self.m, self.k, self.n_list = m, k, n_list

    def add(self, id: str, vector) -> None:  # IvfPq.Add does not validate (:37-45)
        self._write(self._L.pyr_index_add, [id], self._vec(vector))

    def upsert(self, id: str, vector) -> None:
        self.add(id, vector)

    def delete(self, id: str) -> bool:
        lab = self._label_of.get(id)
        if lab is None:
            return False
        labels = np.array([lab], np.int64)
        removed = np.zeros(1, np.uint8)
        check(self._L.pyr_index_remove(self._h, ptr(labels, C.c_int64), 1, ptr(removed, C.c_uint8)))
        return bool(removed[0])

    def pq_state(self):
        ks = C.c_int32()
        check(self._L.pyr_index_pq_state(self._h, None, C.byref(ks), None))
        off, labels, live = self.ivf_layout()
        cb = np.zeros((self.m, ks.value, self.dimension // self.m), np.float32)
        codes = np.zeros((len(labels), self.m), np.uint8)
        check(self._L.pyr_index_pq_state(self._h, ptr(cb, C.c_float), C.byref(ks), ptr(codes, C.c_uint8)))
        return cb, codes, off, labels, live

    def set_codebooks(self, codebooks: np.ndarray) -> None:
        """Supply trained ProductQuantizer codebooks (m x ksub x dim/m) with set_centroids(); the next
        build() then assigns and encodes only, streaming the buffer (pyr_index_set_codebooks)."""
        cb = np.ascontiguousarray(codebooks, dtype=np.float32)
        if cb.ndim != 3 or cb.shape[0] != self.m or cb.shape[2] != self.dimension // self.m:
            raise ArgumentException("codebooks must be m x ksub x dimension/m")
        check(self._L.pyr_index_set_codebooks(self._h, ptr(cb, C.c_float), cb.shape[0], cb.shape[1]))


class DeltaVectorIndex(IVectorIndex, ICentroidsProvider):
    """LSM head/tail composite (DeltaVectorIndex.cs) -- host logic, unchanged from the reference."""

    def __init__(self, head: IVectorIndex, tail: IVectorIndex):
        if head.dimension != tail.dimension:
            raise ArgumentException("Head and Tail dimensions must match")
        if head.metric != tail.metric:
            raise ArgumentException("Head and Tail metrics must match")
        self.head, self.tail = head, tail
        self.dimension, self.metric = head.dimension, head.metric
        self._lock = threading.RLock()  # the reference's ReaderWriterLockSlim (:11); writes and builds exclusive

    def add(self, id, vector):  # :29-43 writes go to the head
        with self._lock:
            self.head.add(id, vector)

    def upsert(self, id, vector):
        with self._lock:
            self.head.upsert(id, vector)

    def delete(self, id) -> bool:  # :58-74
        with self._lock:
            h = self.head.delete(id)
            t = self.tail.delete(id)
            return h or t

    def search(self, query, top_k, options=None):  # :76-122
        with self._lock:
            head_res = self.head.search(query, top_k, options)
            tail_res = self.tail.search(query, top_k, options)
        merged: Dict[str, SearchResult] = {}
        for r in tail_res:
            merged[r.id] = r
        for r in head_res:  # head wins on id collision
            merged[r.id] = r
        out = sorted(merged.values(), key=lambda r: -r.score)
        return out[:top_k]

    def build(self):  # :124-158 compaction head -> tail
        with self._lock:
            items = self.head.scan() if isinstance(self.head, BruteForceVectorIndex) else None
            if items:
                if isinstance(self.tail, (IvfFlatVectorIndex, IvfPqVectorIndex)):
                    # IVF Add == buffer upsert and cannot fail per item: one batched call, then one
                    # batched tombstone pass over the head (same end state as the per-item loop)
                    self.tail.add_batch([i for i, _ in items], np.stack([v for _, v in items]))
                    self.head.delete_many([i for i, _ in items])
                else:
                    for id, vec in items:  # a BruteForce tail throws on a duplicate mid-loop, like the reference
                        self.tail.add(id, vec)
                        self.head.delete(id)
            self.head.build()
            self.tail.build()

    def get_stats(self) -> IndexStats:  # :209-221
        h, t = self.head.get_stats(), self.tail.get_stats()
        return IndexStats(h.count + t.count, h.dimension, h.metric)

    def snapshot(self, path: str) -> None:  # :160-191
        with self._lock:
            head_path, tail_path = path + ".head", path + ".tail"
            self.head.snapshot(head_path + ".tmp")  # both components to temporary paths
            self.tail.snapshot(tail_path + ".tmp")
            for final in (head_path, tail_path):  # then moved into place (with the shim's id maps)
                os.replace(final + ".tmp", final)
                os.replace(final + ".tmp.ids", final + ".ids")
            tmp = path + ".tmp"
            with open(tmp, "w") as f:
                f.write('{"Type": "Delta", "Head": ".head", "Tail": ".tail"}')
            os.replace(tmp, path)  # the manifest last

    def load(self, path: str) -> None:  # :193-212
        with self._lock:
            if os.path.exists(path + ".head"):
                self.head.load(path + ".head")
            if os.path.exists(path + ".tail"):
                self.tail.load(path + ".tail")

    def get_centroids(self):  # :223-233
        return self.tail.get_centroids() if isinstance(self.tail, ICentroidsProvider) else None


class VectorIndexRegistry:
    """Factory branch of Services/VectorIndexRegistry.cs:81-113 with the GPU-backed tail."""

    def __init__(self, device: int = 0):
        self._indices: Dict[str, DeltaVectorIndex] = {}
        self._epochs: Dict[str, int] = {}
        self.device = device

    @staticmethod
    def _int_param(params: Optional[dict], key: str, default: int) -> int:  # GetIntParam :115-126
        """Parameters come from JSON (JsonElement): a number -> GetInt32 (FormatException unless an
        integral int32); a string -> int.TryParse (optional sign, surrounding whitespace); anything else -> default."""
        if params and key in params:
            v = params[key]
            if isinstance(v, bool):  # JsonValueKind.True/False is not Number
                return default
            if isinstance(v, (int, float)):  # a JSON number: JsonElement.GetInt32 throws unless integral int32
                if isinstance(v, float) and not v.is_integer() or not -2**31 <= v < 2**31:
                    raise FormatException(f"The JSON value could not be converted to System.Int32: {v}")
                return int(v)
            if isinstance(v, str):
                m = re.fullmatch(r"\s*([+-]?[0-9]+)\s*", v)
                if m and -2**31 <= int(m.group(1)) < 2**31:
                    return int(m.group(1))
        return default

    def create(self, dimension: int, metric: VectorMetric, algorithm: Optional[str] = None,
               parameters: Optional[dict] = None) -> DeltaVectorIndex:
        algo = (algorithm or "IVF_FLAT").upper()  # :87
        if algo == "HNSW":
            raise InvalidOperationException("HNSW is outside the GPU scan path (SURVEY.md 2, row 12)")
        if algo == "IVF_PQ":  # :96-102
            tail: IVectorIndex = IvfPqVectorIndex(dimension, metric, m=self._int_param(parameters, "m", 4),
                                                  k=self._int_param(parameters, "k", 256),
                                                  n_list=self._int_param(parameters, "nlist", 100),
                                                  device=self.device)
        else:  # :103-108 (unknown strings -> IVF_FLAT)
            tail = IvfFlatVectorIndex(dimension, metric, n_list=self._int_param(parameters, "nlist", 100),
                                      device=self.device)
            nprobe = self._int_param(parameters, "nprobe", 0)
            if nprobe > 0:
                tail.combine_nprobe = nprobe
        head = BruteForceVectorIndex(dimension, metric, device=self.device)  # :111
        return DeltaVectorIndex(head, tail)

    def get_or_create(self, tenant: str, index: str, dimension: int, metric: VectorMetric,
                      algorithm: Optional[str] = None, parameters: Optional[dict] = None) -> DeltaVectorIndex:
        key = f"{tenant}:{index}"
        if key not in self._indices:
            self._indices[key] = self.create(dimension, metric, algorithm, parameters)
        idx = self._indices[key]
        if idx.dimension != dimension:
            raise ArgumentException("Vector dimension mismatch.")
        if idx.metric != metric:
            raise ArgumentException("Vector metric mismatch.")
        return idx

    def try_get_index(self, tenant: str, index: str) -> Optional[DeltaVectorIndex]:
        return self._indices.get(f"{tenant}:{index}")

    def increment_epoch(self, tenant: str, index: str) -> int:  # :52-59
        key = f"{tenant}:{index}"
        if key not in self._indices:
            return 0
        self._epochs[key] = self._epochs.get(key, 0) + 1
        return self._epochs[key]

    def get_epoch(self, tenant: str, index: str) -> int:  # :61-68
        return self._epochs.get(f"{tenant}:{index}", 0)

    def clear(self) -> None:  # :70-73
        self._indices.clear()
        self._epochs.clear()


def kmeans_train(data: np.ndarray, k: int, metric: VectorMetric, max_iter: int = 10, seed: int = 42,
                 device: int = 0) -> np.ndarray:
    """KMeansUtils.Train (KMeansUtils.cs:10-68) on the GPU (pyr_kmeans_train)."""
    x = np.ascontiguousarray(data, dtype=np.float32)
    n, dim = x.shape
    out = np.zeros((max(1, min(max(k, 1), max(n, 1))), dim), np.float32)
    used = C.c_int32()
    check(_lib.load().pyr_kmeans_train(device, ptr(x, C.c_float), n, dim, k, int(metric), max_iter, seed,
                                       ptr(out, C.c_float), C.byref(used)))
    return out[: used.value]


def assign(centroids: np.ndarray, x: np.ndarray, metric: VectorMetric, device: int = 0) -> np.ndarray:
    """KMeansUtils.FindNearestCentroid (KMeansUtils.cs:70-93) of every row of x on the GPU (pyr_assign):
    the list IvfFlatVectorIndex.Build puts it in (ties -> lowest index)."""
    c = np.ascontiguousarray(centroids, dtype=np.float32)
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1, c.shape[1])
    out = np.empty(x.shape[0], np.int32)
    check(_lib.load().pyr_assign(device, ptr(c, C.c_float), c.shape[0], ptr(x, C.c_float), x.shape[0], c.shape[1],
                                 int(metric), ptr(out, C.c_int32)))
    return out


def scalar_quantize(x: np.ndarray, device: int = 0) -> np.ndarray:
    """ScalarQuantizer.Quantize (ScalarQuantizer.cs:23-62) of each row, on the GPU."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    x2 = x.reshape(-1, x.shape[-1])
    out = np.zeros(x2.shape, np.uint8)
    check(_lib.load().pyr_scalar_quantize(device, ptr(x2, C.c_float), x2.shape[0], x2.shape[1], ptr(out, C.c_uint8)))
    return out.reshape(x.shape)


def generate_synthetic(count: int, dim: int, seed: int) -> np.ndarray:
    """Pyrope.Benchmarks GenerateRandomVectors (Program.cs:251-263), via the library."""
    out = np.empty((count, dim), np.float32)
    check(_lib.load().pyr_generate_synthetic(count, dim, seed, ptr(out, C.c_float)))
    return out


BLOCK_ROWS = 65536  # rows per generator block (generate_synthetic_blocked)


def generate_synthetic_blocked(row0: int, count: int, dim: int, seed: int, block_rows: int = BLOCK_ROWS) -> np.ndarray:
    """Rows [row0, row0 + count) of the row-blocked synthetic set: block b (block_rows rows) is the
    Program.cs:251-263 sequence of Random(seed + b) (SURVEY.md 8(d) large-N deviation)."""
    out = np.empty((count, dim), np.float32)
    check(_lib.load().pyr_generate_synthetic_blocked(row0, count, dim, seed, block_rows, ptr(out, C.c_float)))
    return out


class ScalarQuantizer:
    """Vector/ScalarQuantizer.cs (static class): per-vector min/max 8-bit quantization, on the GPU."""

    @staticmethod
    def quantize(vector, device: int = 0):
        """Quantize(float[] vector, out min, out max) (:8-20) -> (codes, min, max); empty -> ([], 0, 0)."""
        if vector is None or len(vector) == 0:
            return np.zeros(0, np.uint8), 0.0, 0.0
        v = np.ascontiguousarray(vector, dtype=np.float32).reshape(1, -1)
        codes = np.zeros(v.shape, np.uint8)
        mn, mx = np.zeros(1, np.float32), np.zeros(1, np.float32)
        check(_lib.load().pyr_scalar_quantize_minmax(device, ptr(v, C.c_float), 1, v.shape[1], ptr(codes, C.c_uint8),
                                                     ptr(mn, C.c_float), ptr(mx, C.c_float)))
        return codes[0], float(mn[0]), float(mx[0])

    @staticmethod
    def quantize_into(vector, destination: np.ndarray, device: int = 0):
        """Quantize(ReadOnlySpan<float>, Span<byte>, out min, out max) (:22-62) -> (min, max)."""
        if len(vector) != len(destination):
            raise ArgumentException("Vector and destination lengths must match.")
        if len(vector) == 0:
            return 0.0, 0.0
        codes, mn, mx = ScalarQuantizer.quantize(vector, device)
        destination[:] = codes
        return mn, mx

    @staticmethod
    def dequantize(codes, vmin: float, vmax: float, device: int = 0) -> np.ndarray:
        """Dequantize(byte[], min, max) (:64-84)."""
        if codes is None:
            return np.zeros(0, np.float32)
        c = np.ascontiguousarray(codes, dtype=np.uint8).reshape(1, -1)
        out = np.zeros(c.shape, np.float32)
        if c.shape[1] == 0:
            return out[0]
        mn, mx = np.array([vmin], np.float32), np.array([vmax], np.float32)
        check(_lib.load().pyr_scalar_dequantize(device, ptr(c, C.c_uint8), 1, c.shape[1], ptr(mn, C.c_float),
                                                ptr(mx, C.c_float), ptr(out, C.c_float)))
        return out[0]
