"""TFRecord files and ``tf.train.Example`` records of the dataset path, without TensorFlow.

Restates what the reference's data path reads and writes:
* framing (``tf.data.TFRecordDataset`` / ``tf.python_io.TFRecordWriter``, used by
  datasets/ljspeech/dataset.py:96-112 and utils/tfrecord.py:46-49): ``uint64 length |
  uint32 masked_crc32c(length) | payload | uint32 masked_crc32c(payload)``.  Framing, CRC-32C and
  record indexing run in libsat_hip's host entries (``sat_tfrecord_frame`` /
  ``sat_tfrecord_index``, csrc/records.hip);
* the ``tf.train.Example`` protobuf wire format (``Example{features=1}``, ``Features{map<string,
  Feature> feature=1}``, ``Feature{bytes_list=1 | float_list=2 | int64_list=3}``, each list a
  repeated field 1, packed or not), encoded and decoded here;
* the LJSpeech record types of preprocess/ljspeech.py:23-45: source records ``id, key,
  source (int64 bytes), source_length, text`` and target records ``id, key, mel (float32
  bytes), target_length, mel_width``; parsed as ``parse_preprocessed_source_data`` /
  ``decode_preprocessed_source_data`` (datasets/ljspeech/dataset.py:53-73) and the mel
  analogues the dataset imports from utils.tfrecord (``PreprocessedMelData``).
"""

from __future__ import annotations

import ctypes
import struct
from collections import namedtuple
from typing import Dict, Iterable, Iterator, List, Tuple, Union

import numpy as np

from . import _lib


class PreprocessedSourceData(namedtuple("PreprocessedSourceData",
                                        ["id", "key", "source", "source_length", "text"])):
    pass


class PreprocessedMelData(namedtuple("PreprocessedMelData",
                                     ["id", "key", "mel", "target_length", "mel_width"])):
    pass


Feature = Tuple[str, list]          # ("int64" | "bytes" | "float", values)


# ---------------------------------------------------------------- framing (libsat_hip host)
def frame_record(payload: bytes) -> bytes:
    out = ctypes.create_string_buffer(len(payload) + 16)
    n = _lib.load().sat_tfrecord_frame(payload, len(payload), out)
    return out.raw[:n]


def split_records(buf: bytes, verify: bool = True) -> List[bytes]:
    """Payloads of a buffer of concatenated TFRecords (checksums verified by default)."""
    L = _lib.load()
    cap = max(1, len(buf) // 16)
    spans = (ctypes.c_int64 * (2 * cap))()
    n = L.sat_tfrecord_index(buf, len(buf), int(verify), spans, cap)
    if n < 0:
        raise ValueError("corrupt TFRecord data: " + L.sat_last_error_string().decode(errors="replace"))
    return [buf[spans[2 * i]: spans[2 * i] + spans[2 * i + 1]] for i in range(n)]


def write_tfrecords(records: Iterable[bytes], filename: str) -> None:
    with open(filename, "wb") as f:
        for r in records:
            f.write(frame_record(r))


def read_tfrecords(filename: str, verify: bool = True) -> Iterator[bytes]:
    with open(filename, "rb") as f:
        buf = f.read()
    yield from split_records(buf, verify)


# ---------------------------------------------------------------- protobuf wire format
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1                 # int64 two's complement, as protobuf
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        if i >= len(b):
            raise ValueError("truncated varint")
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _ld(field: int, payload: bytes) -> bytes:
    return _varint(field << 3 | 2) + _varint(len(payload)) + payload


def _fields(b: bytes) -> Iterator[Tuple[int, int, Union[int, bytes]]]:
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 2:
            n, i = _read_varint(b, i)
            if i + n > len(b):
                raise ValueError("truncated length-delimited field")
            v, i = b[i:i + n], i + n
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield field, wt, v


def encode_example(features: Dict[str, Feature]) -> bytes:
    """``tf.train.Example(features=tf.train.Features(feature=...)).SerializeToString()``;
    map entries in the given order, numeric lists packed (proto3)."""
    entries = b""
    for name, (kind, values) in features.items():
        if kind == "bytes":
            lst = b"".join(_ld(1, bytes(v)) for v in values)
            feat = _ld(1, lst)
        elif kind == "float":
            feat = _ld(2, _ld(1, np.asarray(values, "<f4").tobytes()) if len(values) else b"")
        elif kind == "int64":
            feat = _ld(3, _ld(1, b"".join(_varint(int(v)) for v in values)) if len(values) else b"")
        else:
            raise ValueError(f"unknown feature kind {kind!r}")
        entries += _ld(1, _ld(1, name.encode("utf-8")) + _ld(2, feat))
    return _ld(1, entries)


def decode_example(buf: bytes) -> Dict[str, Feature]:
    out: Dict[str, Feature] = {}
    for f, wt, feats in _fields(buf):
        if f != 1 or wt != 2:
            continue
        for f2, wt2, entry in _fields(feats):
            if f2 != 1 or wt2 != 2:
                continue
            name, feat = "", b""
            for f3, _, v in _fields(entry):
                if f3 == 1:
                    name = v.decode("utf-8")
                elif f3 == 2:
                    feat = v
            kind, values = "bytes", []
            for f4, _, lst in _fields(feat):
                if f4 == 1:
                    kind, values = "bytes", [v for f5, _, v in _fields(lst) if f5 == 1]
                elif f4 == 2:
                    kind, values = "float", []
                    for f5, wt5, v in _fields(lst):
                        if f5 == 1:
                            values.extend(np.frombuffer(v, "<f4").tolist() if wt5 == 2
                                          else [struct.unpack("<f", v)[0]])
                elif f4 == 3:
                    kind, values = "int64", []
                    for f5, wt5, v in _fields(lst):
                        if f5 != 1:
                            continue
                        if wt5 == 2:
                            j = 0
                            while j < len(v):
                                x, j = _read_varint(v, j)
                                values.append(x - (1 << 64) if x >> 63 else x)
                        else:
                            values.append(v - (1 << 64) if v >> 63 else v)
            out[name] = (kind, values)
    return out


def _scalar(ex: Dict[str, Feature], name: str, kind: str):
    """tf.FixedLenFeature((), kind): exactly one value, else InvalidArgumentError (ValueError)."""
    if name not in ex:
        raise ValueError(f"Feature: {name} (data type: {kind}) is required but could not be found")
    k, v = ex[name]
    if k != kind or len(v) != 1:
        raise ValueError(f"Key: {name}.  Can't parse serialized Example: expected one {kind}")
    return v[0]


# ---------------------------------------------------------------- LJSpeech record types
def source_example(_id: int, key: str, source: np.ndarray, text: str) -> bytes:
    """preprocess/ljspeech.py:35-45 (write_preprocessed_source_data's Example)."""
    source = np.ascontiguousarray(source, dtype="<i8")
    return encode_example({"id": ("int64", [_id]), "key": ("bytes", [key.encode("utf-8")]),
                           "source": ("bytes", [source.tobytes()]),
                           "source_length": ("int64", [len(source)]),
                           "text": ("bytes", [text.encode("utf-8")])})


def target_example(_id: int, key: str, mel: np.ndarray) -> bytes:
    """preprocess/ljspeech.py:23-32 (write_preprocessed_target_data's Example)."""
    mel = np.ascontiguousarray(mel, dtype="<f4")
    return encode_example({"id": ("int64", [_id]), "key": ("bytes", [key.encode("utf-8")]),
                           "mel": ("bytes", [mel.tobytes()]),
                           "target_length": ("int64", [len(mel)]),
                           "mel_width": ("int64", [mel.shape[1]])})


def write_preprocessed_source_data(_id: int, key: str, source: np.ndarray, text: str,
                                   filename: str) -> None:
    write_tfrecords([source_example(_id, key, source, text)], filename)


def write_preprocessed_target_data(_id: int, key: str, mel: np.ndarray, filename: str) -> None:
    write_tfrecords([target_example(_id, key, mel)], filename)


def parse_preprocessed_source_data(record: bytes) -> PreprocessedSourceData:
    """parse_preprocessed_source_data + decode_preprocessed_source_data
    (datasets/ljspeech/dataset.py:53-73): source = decode_raw(int64)."""
    ex = decode_example(record)
    return PreprocessedSourceData(
        id=_scalar(ex, "id", "int64"), key=_scalar(ex, "key", "bytes"),
        source=np.frombuffer(_scalar(ex, "source", "bytes"), "<i8").astype(np.int64),
        source_length=_scalar(ex, "source_length", "int64"), text=_scalar(ex, "text", "bytes"))


def parse_preprocessed_mel_data(record: bytes) -> PreprocessedMelData:
    """The mel target record (preprocess/ljspeech.py:23-32): mel = decode_raw(float32)
    reshaped [target_length, mel_width]."""
    ex = decode_example(record)
    width = _scalar(ex, "mel_width", "int64")
    mel = np.frombuffer(_scalar(ex, "mel", "bytes"), "<f4").astype(np.float32)
    if width <= 0 or mel.size % width:
        raise ValueError(f"mel record: {mel.size} floats do not fill rows of width {width}")
    return PreprocessedMelData(id=_scalar(ex, "id", "int64"), key=_scalar(ex, "key", "bytes"),
                               mel=mel.reshape(-1, width),
                               target_length=_scalar(ex, "target_length", "int64"),
                               mel_width=width)
