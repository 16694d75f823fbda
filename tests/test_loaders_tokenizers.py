"""Token shards, batch loader, downloader and tokenizer wrapper (CPU, no network)."""
import os
import sys
import types
from unittest.mock import MagicMock, patch

import numpy as np
import pytest

from penroz.utils import loaders
from penroz.utils.loaders import Downloader, Loader


def test_next_batch_semantics(workdir):
    loaders.save_shard("ds", 0, list(range(10)), 100)
    loaders.save_shard("ds", 1, list(range(10, 20)), 100)
    loaders.save_shard("ds_extra", 0, [99] * 10, 100)  # substring match must not pick this up
    ld = Loader("ds", 0, begin_idx=0, buffer_size=4, idx_offset=4)
    assert ld.list() == ["ds_000000.npy", "ds_000001.npy"]
    x, y = ld.next_batch()
    assert list(x) == [0, 1, 2, 3] and list(y) == [1, 2, 3, 4]
    x, y = ld.next_batch()
    assert list(x) == [4, 5, 6, 7]
    x, y = ld.next_batch()  # crosses into shard 1
    assert list(x) == [8, 9, 10, 11] and list(y) == [9, 10, 11, 12]
    x, t = ld.next_batch(target_offset=0)
    assert t is None and len(x) == 4


def test_wraparound_and_rank_stride(workdir):
    loaders.save_shard("w", 0, list(range(6)), 100)
    r1 = Loader("w", 0, begin_idx=2, buffer_size=2, idx_offset=4)
    assert list(r1.next_batch()[0]) == [2, 3]
    assert list(r1.next_batch()[0]) == [0, 1]  # wrapped to the (only) shard


def test_large_vocab_uses_uint32(workdir):
    p = loaders.save_shard("big", 0, [70000, 1], 262144)
    assert np.load(p).dtype == np.uint32
    p = loaders.save_shard("small", 0, [5, 1], 50257)
    assert np.load(p).dtype == np.uint16


def test_delete(workdir):
    loaders.synthetic_shards("d", 2, 10, 50)
    Loader("d").delete()
    assert Loader("d").list() == []


def test_downloader_small_shards_and_multiprocess_tokenise(workdir):
    fake_tok = MagicMock()
    fake_tok.tokenize.side_effect = lambda t: [len(t)] * 3
    fake_tok.vocab_size = 100
    with patch("penroz.utils.tokenizers.Tokenizer", return_value=fake_tok):
        d = Downloader("dl", 5, "hf-name")
    pool = MagicMock()
    pool.__enter__.return_value.imap.side_effect = lambda f, it, chunksize: map(f, it)
    fake_datasets = types.SimpleNamespace(load_dataset=lambda *a, **k: {"text": ["ab", "abc", "abcd"]})
    with patch.dict(sys.modules, {"datasets": fake_datasets}), patch("multiprocessing.Pool", return_value=pool):
        d.download("p", "n", "train")  # shard_size < 100 divided by zero in the reference (bug 13)
    files = Loader("dl").list()
    assert files == ["dl_000000.npy", "dl_000001.npy"]
    assert list(np.load(os.path.join(loaders.DATA_FOLDER, files[0]))) == [2, 2, 2, 3, 3]


def test_tokenizer_hf_and_pickle():
    from penroz.utils import tokenizers
    enc = MagicMock()
    enc.encode.return_value = [5, 6]
    enc.eos_token_id = 0
    enc.decode.return_value = "hi"
    enc.vocab_size = 10
    with patch("transformers.AutoTokenizer.from_pretrained", return_value=enc):
        t = tokenizers.Tokenizer("some/model")
        assert t.tokenize("hi") == [5, 6, 0]
        assert t.decode([5, 6]) == "hi"
        import pickle
        t2 = pickle.loads(pickle.dumps(t))
        assert t2.tokenize("x") == [5, 6, 0]


def test_tokenizer_tiktoken():
    from penroz.utils import tokenizers
    fake = types.ModuleType("tiktoken")
    enc = MagicMock()
    enc.encode_ordinary.return_value = [1, 2]
    enc.eot_token = 50256
    enc.n_vocab = 50257
    enc.decode.return_value = "ok"
    fake.get_encoding = lambda name: enc
    with patch.dict(sys.modules, {"tiktoken": fake}):
        t = tokenizers.Tokenizer("tiktoken/gpt2")
        assert t.tokenize("x") == [1, 2, 50256] and t.decode([1]) == "ok"


class _EagerLoader:
    """The reference loader's arithmetic (loaders.py:65-87) on fully materialised int32 shards."""

    def __init__(self, shards, begin_shard, begin_idx, buffer_size, idx_offset):
        self.shards, self.shard_idx = shards, begin_shard
        self.buffer_size, self.idx_offset, self.token_idx = buffer_size, idx_offset, begin_idx
        self.tokens = np.empty((0,), dtype=np.int32)

    def next_batch(self, target_offset=1):
        if len(self.tokens) == 0:
            self.tokens = self.shards[self.shard_idx % len(self.shards)].astype(np.int32)
        for _ in range(len(self.shards)):
            if len(self.tokens) < self.token_idx + self.idx_offset + target_offset:
                self.shard_idx = (self.shard_idx + 1) % len(self.shards)
                self.tokens = np.concatenate((self.tokens[self.token_idx:], self.shards[self.shard_idx].astype(np.int32)))
                self.token_idx = 0
            else:
                break
        i = self.token_idx
        inp = self.tokens[i:i + self.buffer_size]
        tgt = self.tokens[i + target_offset:i + self.buffer_size + target_offset] if target_offset > 0 else None
        self.token_idx += self.idx_offset
        return inp, tgt


@pytest.mark.parametrize("seed", range(12))
def test_mmap_window_loader_matches_eager_semantics(workdir, seed):
    import penroz.utils.loaders as L
    rng = np.random.default_rng(seed)
    nsh = int(rng.integers(1, 4))
    sizes = [int(rng.integers(20, 120)) for _ in range(nsh)]
    arrs = [rng.integers(0, 70000 if seed % 2 else 500, n) for n in sizes]
    for i, a in enumerate(arrs):
        L.save_shard(f"w{seed}", i, a, 70000 if seed % 2 else 500)
    buf = int(rng.integers(4, 24))
    world = int(rng.integers(1, 3))
    rank = int(rng.integers(0, world))
    tofs = int(rng.integers(0, 2))
    got = L.Loader(f"w{seed}", 0, buf * rank, buf, buf * world)
    assert isinstance(got._load(), np.memmap)
    ref = _EagerLoader([np.asarray(a) for a in arrs], 0, buf * rank, buf, buf * world)
    for _ in range(25):
        gi, gt = got.next_batch(tofs)
        ri, rt = ref.next_batch(tofs)
        assert gi.dtype == np.int32 and np.array_equal(gi, ri)
        assert (gt is None and rt is None) or np.array_equal(gt, rt)
