""".diskann v2 index files (+ optional SQ8 trailer) — the on-disk input of the DiskProvider path.

Layout (rust_lib/src/file_format.rs:3-18, writer :84-120), little endian:
  [0:4]   magic "DANN"       [4:8]  version u32 = 2      [8:12]  num_vectors u32
  [12:16] dimension u32      [16:20] max_degree u32      [20:24] num_entry_points u32
  [24]    metric u8 (0=L2, 1=IP), [25:28] pad             [28:32] build_complexity u32
  entry point ids   num_entry_points × u32
  vectors           num_vectors × dimension × f32
  adjacency         num_vectors × max_degree × u32 (unused slots = u32::MAX)
SQ8 trailer (index_manager.rs:513-533 writer, :629-668 reader), directly after the adjacency:
  "SQ8\\0", dim u32, qlen u64, min[dim] f32, scale[dim] f32, codes[qlen] u8

``open_index`` validates like DiskProvider::open (disk_provider.rs:201-279): magic, version, and
``len >= expected`` only (so a trailer is tolerated), and memory-maps the segments.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import numpy as np

MAGIC = b"DANN"
VERSION = 2
HEADER_SIZE = 32
SQ8_MARKER = b"SQ8\0"


@dataclass
class DiskannFile:
    num_vectors: int
    dimension: int
    max_degree: int
    metric: int
    build_complexity: int
    entry_points: np.ndarray          # u32
    vectors: np.ndarray               # (N, d) f32 (memory-mapped)
    adjacency: np.ndarray             # (N, R) u32 (memory-mapped)
    sq8_min: Optional[np.ndarray] = None
    sq8_scale: Optional[np.ndarray] = None
    sq8_codes: Optional[np.ndarray] = None  # (N, d) u8

    def neighbors(self, i: int) -> np.ndarray:
        """get_neighbors (disk_provider.rs:317-332): trim at the first u32::MAX."""
        row = self.adjacency[i]
        stop = np.nonzero(row == 0xFFFFFFFF)[0]
        return row[: stop[0]] if len(stop) else row


def write_index(path, vectors: np.ndarray, adjacency: np.ndarray, entry_points, metric: int = 0,
                build_complexity: int = 128, sq8: Optional[tuple] = None) -> None:
    """file_format.rs::write_index (+ the SQ8 trailer of InMemoryIndex::serialize_to_bytes)."""
    vectors = np.ascontiguousarray(vectors, np.float32)
    adjacency = np.ascontiguousarray(adjacency, np.uint32)
    eps = np.ascontiguousarray(entry_points, np.uint32)
    n, d = vectors.shape
    r = adjacency.shape[1]
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<IIIII", VERSION, n, d, r, len(eps)))
        f.write(struct.pack("<B3xI", metric, build_complexity))
        f.write(eps.tobytes())
        f.write(vectors.tobytes())
        f.write(adjacency.tobytes())
        if sq8 is not None:
            mins, scale, codes = sq8
            codes = np.ascontiguousarray(codes, np.uint8)
            f.write(SQ8_MARKER)
            f.write(struct.pack("<IQ", d, codes.size))
            f.write(np.ascontiguousarray(mins, np.float32).tobytes())
            f.write(np.ascontiguousarray(scale, np.float32).tobytes())
            f.write(codes.tobytes())


def open_index(path) -> DiskannFile:
    p = Path(path)
    mm = np.memmap(p, dtype=np.uint8, mode="r")
    if len(mm) < HEADER_SIZE:
        raise ValueError("file too small")
    if bytes(mm[:4]) != MAGIC:
        raise ValueError("invalid magic bytes")
    version, n, d, r, n_ep = struct.unpack("<IIIII", bytes(mm[4:24]))
    if version != VERSION:
        raise ValueError(f"unsupported version {version} (expected {VERSION})")
    metric = int(mm[24])
    (build_complexity,) = struct.unpack("<I", bytes(mm[28:32]))
    ep_off = HEADER_SIZE
    vec_off = ep_off + 4 * n_ep
    adj_off = vec_off + 4 * n * d
    end = adj_off + 4 * n * r
    if len(mm) < end:
        raise ValueError(f"file too small: expected {end} bytes, got {len(mm)}")
    eps = np.frombuffer(mm, np.uint32, n_ep, ep_off).copy()
    vecs = np.frombuffer(mm, np.float32, n * d, vec_off).reshape(n, d)
    adj = np.frombuffer(mm, np.uint32, n * r, adj_off).reshape(n, r)
    out = DiskannFile(n, d, r, 1 if metric == 1 else 0, build_complexity, eps, vecs, adj)
    if len(mm) > end + 4 and bytes(mm[end:end + 4]) == SQ8_MARKER:
        sq_dim, qlen = struct.unpack("<IQ", bytes(mm[end + 4:end + 16]))
        po = end + 16
        total = po + 8 * sq_dim + qlen
        if total > len(mm):
            raise ValueError(f"SQ8 section truncated: need {total} bytes, have {len(mm)}")
        out.sq8_min = np.frombuffer(mm, np.float32, sq_dim, po).copy()
        out.sq8_scale = np.frombuffer(mm, np.float32, sq_dim, po + 4 * sq_dim).copy()
        out.sq8_codes = np.frombuffer(mm, np.uint8, qlen, po + 8 * sq_dim).reshape(-1, sq_dim)
    return out
