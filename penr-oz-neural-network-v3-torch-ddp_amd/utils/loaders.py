"""Token shards: download/tokenise to ``.npy`` shards, and the rank-strided batch loader.

Parity with the reference (``loaders.py:12-87``): shards ``data/{dataset_id}_{NNNNNN}.npy``,
``Loader(dataset_id, begin_shard, begin_idx, buffer_size, idx_offset).next_batch(target_offset)``
with shard roll-over/wrap-around, ``list()``, ``delete()``.

Fixes / MI355X-first changes:
  * shards are matched exactly (``{id}_NNNNNN.npy``), not by substring (bug 11);
  * uint16 is used only while the vocabulary fits, else uint32 (bug 12: Gemma's 262k vocab);
  * progress logging never divides by zero for small shards (bug 13);
  * ``target_offset=0`` returns the same ``(input, target)`` tuple shape (targets may come from
    a second loader; the reference's evaluate path crashed on it — bug 1);
  * shards are memory-mapped (``mmap_mode='r'``) and never converted whole: the loader keeps a
    view of (the unread tail of the previous shard, the current shard) and converts only each
    batch window to int32, so a rank touches the pages it reads and nothing more;
  * :func:`synthetic_shards` writes uniform-random shards for benchmarks/tests (no network).
"""
from __future__ import annotations

import logging
import multiprocessing
import os
import re
from typing import Tuple

import numpy as np

log = logging.getLogger(__name__)

DATA_FOLDER = os.environ.get("PENROZ_DATA_FOLDER", "data")
num_procs = max(1, (os.cpu_count() or 2) // 2)


def _shard_regex(dataset_id: str):
    return re.compile(rf"^{re.escape(dataset_id)}_(\d{{6}})\.npy$")


def shard_dtype(vocab_size: int | None, tokens=None):
    hi = vocab_size if vocab_size is not None else (int(max(tokens)) + 1 if tokens is not None and len(tokens) else 0)
    return np.uint16 if hi <= 65536 else np.uint32


def save_shard(dataset_id: str, shard_idx: int, tokens, vocab_size: int | None = None) -> str:
    os.makedirs(DATA_FOLDER, exist_ok=True)
    path = os.path.join(DATA_FOLDER, f"{dataset_id}_{shard_idx:06d}")
    np.save(path, np.asarray(tokens, dtype=shard_dtype(vocab_size, tokens)))
    log.info(f"Saved shard {shard_idx:06d} with {len(tokens)} tokens into {path}")
    return path + ".npy"


def synthetic_shards(dataset_id: str, num_shards: int, shard_size: int, vocab_size: int, seed: int = 0) -> list[str]:
    rng = np.random.default_rng(seed)
    return [save_shard(dataset_id, i, rng.integers(0, vocab_size, shard_size), vocab_size) for i in range(num_shards)]


class Downloader:
    """HF dataset -> tokenised shards of ``shard_size`` tokens (multiprocess tokenisation)."""

    def __init__(self, dataset_id: str, shard_size: int, encoding: str):
        from penroz.utils.tokenizers import Tokenizer
        self.dataset_id = dataset_id
        self.shard_size = int(shard_size)
        self.encoding = encoding
        self.tokenizer = Tokenizer(encoding)

    def _save(self, shard_idx: int, tokens: list[int]):
        save_shard(self.dataset_id, shard_idx, tokens, getattr(self.tokenizer, "vocab_size", None))

    def download(self, path: str, name: str, split: str):
        from datasets import load_dataset
        ds = load_dataset(path, name, split=split)
        log_every = max(1, self.shard_size // 100)
        with multiprocessing.Pool(num_procs) as pool:
            tokens: list[int] = []
            shard_idx = 0
            for i, chunk in enumerate(pool.imap(self.tokenizer.tokenize, ds["text"], chunksize=16)):
                tokens.extend(chunk)
                while len(tokens) >= self.shard_size:
                    self._save(shard_idx, tokens[:self.shard_size])
                    shard_idx += 1
                    tokens = tokens[self.shard_size:]
                if i % log_every == 0:
                    log.info(f"Cached {len(tokens)} of {self.shard_size} tokens in shard {shard_idx:06d}")
            if tokens:
                self._save(shard_idx, tokens)


class Loader:
    def __init__(self, dataset_id: str, begin_shard: int = 0, begin_idx: int = 0, buffer_size: int = 0,
                 idx_offset: int = 0):
        from penroz.parallel.dist import master_proc
        rx = _shard_regex(dataset_id)
        files = os.listdir(DATA_FOLDER) if os.path.isdir(DATA_FOLDER) else []
        self.shards = sorted(f for f in files if rx.match(f))
        if master_proc():
            log.info(f"Found {len(self.shards)} shard(s) for {dataset_id}")
        self.shard_idx = begin_shard
        self.buffer_size = buffer_size
        self.idx_offset = idx_offset
        self.token_idx = begin_idx
        self.tokens = _Window([])

    def list(self) -> list[str]:
        return self.shards

    def delete(self):
        for shard in self.shards:
            os.remove(os.path.join(DATA_FOLDER, shard))

    def _load(self) -> np.ndarray:
        """The current shard as a read-only memory map (uint16/uint32 on disk, not converted)."""
        if not self.shards:
            raise KeyError("no shards found for dataset")
        return np.load(os.path.join(DATA_FOLDER, self.shards[self.shard_idx % len(self.shards)]), mmap_mode="r")

    def next_batch(self, target_offset: int = 1) -> Tuple[np.ndarray, np.ndarray | None]:
        """Reference semantics (``loaders.py:65-87``): input = tokens[i : i+buffer], target shifted
        by ``target_offset``, advance by ``idx_offset``; when the window would run past the
        buffered tokens, the unread tail is carried over and the next shard appended (wrapping)."""
        if len(self.tokens) == 0:
            self.tokens = _Window([self._load()])
        for _ in range(max(1, len(self.shards))):
            if len(self.tokens) < self.token_idx + self.idx_offset + target_offset:
                self.shard_idx = (self.shard_idx + 1) % len(self.shards)
                self.tokens = _Window(self.tokens.tail(self.token_idx) + [self._load()])
                self.token_idx = 0
            else:
                break
        i = self.token_idx
        inp = self.tokens.slice(i, i + self.buffer_size)
        tgt = None
        if target_offset > 0:
            tgt = self.tokens.slice(i + target_offset, i + self.buffer_size + target_offset)
        self.token_idx += self.idx_offset
        return inp, tgt


class _Window:
    """A logical concatenation of 1-D arrays (memory maps or views) without copying them."""

    def __init__(self, parts: list[np.ndarray]):
        self.parts = [p for p in parts if len(p)]
        self.n = sum(len(p) for p in self.parts)

    def __len__(self) -> int:
        return self.n

    def tail(self, start: int) -> list[np.ndarray]:
        """Views of everything from ``start`` on."""
        out = []
        for p in self.parts:
            if start >= len(p):
                start -= len(p)
                continue
            out.append(p[start:])
            start = 0
        return out

    def slice(self, a: int, b: int) -> np.ndarray:
        """tokens[a:b] as int32 (only this window is read from the shard files)."""
        b = min(b, self.n)
        chunks, off = [], 0
        for p in self.parts:
            lo, hi = max(a - off, 0), min(b - off, len(p))
            if lo < hi:
                chunks.append(np.asarray(p[lo:hi], dtype=np.int32))
            off += len(p)
            if off >= b:
                break
        if not chunks:
            return np.empty((0,), dtype=np.int32)
        return chunks[0] if len(chunks) == 1 else np.concatenate(chunks)
