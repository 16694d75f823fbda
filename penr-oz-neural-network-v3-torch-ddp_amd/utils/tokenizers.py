"""Tokenizer wrapper (parity with the reference ``gpt_tokenizers.py:1-22``).

``"tiktoken/<encoding>"`` -> tiktoken ``encode_ordinary`` + end-of-text; anything else -> a
HuggingFace ``AutoTokenizer`` (``encode`` without special tokens + EOS).  tiktoken is not
installed in this image; it is imported lazily so the rest of the framework works without it
(the API then returns a clear 400 for tiktoken encodings).  Instances pickle by encoding name,
so they can be shipped to tokenisation worker processes.
"""
from __future__ import annotations

TIKTOKEN_PREFIX = "tiktoken/"


class Tokenizer:
    def __init__(self, encoding_name: str):
        self.encoding_name = encoding_name
        self._build()

    def _build(self):
        name = self.encoding_name
        if name.startswith(TIKTOKEN_PREFIX):
            try:
                import tiktoken
            except ImportError as e:  # pragma: no cover - depends on the image
                raise ValueError(f"tiktoken is not available for encoding {name}") from e
            enc = tiktoken.get_encoding(name[len(TIKTOKEN_PREFIX):])
            self._kind, self._enc = "tiktoken", enc
            self.vocab_size = enc.n_vocab
        else:
            from transformers import AutoTokenizer
            enc = AutoTokenizer.from_pretrained(name)
            self._kind, self._enc = "hf", enc
            self.vocab_size = getattr(enc, "vocab_size", None)

    def __getstate__(self):
        return {"encoding_name": self.encoding_name}

    def __setstate__(self, state):
        self.encoding_name = state["encoding_name"]
        self._build()

    def tokenize(self, text: str) -> list[int]:
        enc = self._enc
        if self._kind == "tiktoken":
            return enc.encode_ordinary(text) + [enc.eot_token]
        eos = [enc.eos_token_id] if enc.eos_token_id is not None else []
        return enc.encode(text, add_special_tokens=False) + eos

    def decode(self, tokens: list[int]) -> str:
        return self._enc.decode(tokens)
