"""``SPELayer`` — the reference's tokenizer layer (include/op/encode.h:16-28, source/op/encode.cpp:5-27).

The reference wraps sentencepiece's C++ ``SentencePieceProcessor``; that library is not in this image, but the
Python ``sentencepiece`` package (0.2.x) is, and it is the same processor. Host-only text I/O: the decode path
never sees text, only the token ids this layer produces.

Behaviour kept from the reference:
  * the constructor loads the model file and raises ``RuntimeError`` with the library's status text when
    that fails (encode.cpp:6-10: ``throw std::runtime_error(status.ToString())``);
  * ``encode`` returns the piece ids of the text (encode.cpp:13-17), ``decode`` the text of an id list
    (encode.cpp:19-23), ``GetVocabularySize`` the processor's piece count (encode.cpp:25-27).
"""
from __future__ import annotations


class SPELayer:
    def __init__(self, model_file: str = "", model_proto: bytes | None = None):
        """``model_file``: a sentencepiece ``.model`` path (the reference's only form); ``model_proto``: the same
        bytes in memory (extension, for tests and embedded tokenizers)."""
        try:
            import sentencepiece
        except ImportError as e:  # the reference fails to build without it; here the layer fails to load
            raise RuntimeError(f"sentencepiece is not importable: {e}") from e
        self._sp = sentencepiece.SentencePieceProcessor()
        try:
            if model_proto is not None:
                self._sp.LoadFromSerializedProto(model_proto)
            else:
                self._sp.Load(model_file)
        except (OSError, RuntimeError, TypeError) as e:
            raise RuntimeError(str(e)) from e

    def encode(self, text: str) -> list[int]:
        return [int(i) for i in self._sp.EncodeAsIds(text)]

    def decode(self, ids) -> str:
        return self._sp.DecodeIds([int(i) for i in ids])

    def GetVocabularySize(self) -> int:  # noqa: N802 — the reference's name
        return int(self._sp.GetPieceSize())


def render_predict(layer: SPELayer, fed, last: int) -> str:
    """The text the reference's ``LlamaModel::predict`` writes to stdout (model.cpp:142-187): the first prompt
    token, then one token per forward — the next prompt token while the prompt lasts, the argmax after it —
    each decoded on its own (``decode({id})``) and followed by one space, then a newline. ``fed`` are the tokens
    fed at positions 0..max_length-1, ``last`` the argmax of the final forward (printed, never fed)."""
    return "".join(layer.decode([t]) + " " for t in list(fed) + [last]) + "\n"
