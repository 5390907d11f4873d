"""LJSpeech dataset pipeline over TFRecord files: ``datasets/ljspeech/dataset.py`` without tf.data.

Same classes, methods and record types as the reference:
``DatasetSource.create_from_tfrecord_files(source_files, target_files, hparams, cycle_length,
...)`` (:96-112) -> ``prepare_and_zip()`` (:114-117) -> ``ZippedDataset`` with
``filter_by_max_output_length`` / ``shuffle`` / ``repeat`` / ``shuffle_and_repeat`` / ``cache``
(:185-219) -> ``group_by_batch(batch_size)`` (:237-285) -> ``BatchedDataset`` with ``prefetch``
and ``merge_target_to_source`` (:288-320).  Elements are numpy records; a BatchedDataset
iterates ``(SourceData, MelData)`` batches padded as the reference pads them, which
``model_fn`` takes directly (``MelData.mel`` is the ``codes`` slot, ``spec_loss_mask`` the
code loss mask).

Target preparation (:126-167): ``mel = (mel - average_mel_level_db) / stddev_mel_level_db``;
``r`` frames of ``silence_mel_level_db`` at head and tail; ``target_length + 2r`` rounded up to a
multiple of r with more silence (``(L // r + 1) * r`` when ``L % r != 0``); ``done = [0..0, 1]``
of ``L / r``; ``spec_loss_mask = 1[L]``, ``binary_loss_mask = 1[L / r]``.

Batching (:237-285, tf.contrib.data.group_by_window with window_size = 5 * batch_size): the key
is ``min(num_buckets, min(target_length - approx_min_target_length, 0) // bucket_width)`` --
note ``tf.minimum(.., 0)``: every utterance of ``>= approx_min_target_length`` frames shares
bucket 0 (kept as the reference has it).  A window is emitted as padded batches when it holds
``window_size`` elements; the rest are flushed at the end of the input in order of each key's
first appearance.  Padding: source 0, mel ``silence_mel_level_db``, done 1, masks 0, scalars 0.

Randomness (``shuffle``) uses ``numpy.random.default_rng(seed)`` -- the same buffer algorithm as
tf.data's shuffle (fill ``buffer_size``, emit a uniformly chosen slot, refill it), not its
random stream.
"""

from __future__ import annotations

import queue
import threading
from collections import OrderedDict, namedtuple
from typing import Callable, Iterable, Iterator, List, Optional, Sequence

import numpy as np

from . import tfrecord as R


class SourceData(namedtuple("SourceData", ["id", "key", "source", "source_length", "text"])):
    pass


class MelData(namedtuple("MelData", ["id", "key", "mel", "mel_width", "target_length", "done",
                                     "spec_loss_mask", "binary_loss_mask"])):
    pass


class SourceDataForPrediction(namedtuple("SourceDataForPrediction",
                                         ["id", "key", "source", "source_length", "text", "mel",
                                          "mel_width", "target_length"])):
    pass


class _Dataset:
    """A re-iterable element stream (the role of a tf.data.Dataset here)."""

    def __init__(self, make: Callable[[], Iterator]):
        self._make = make

    def __iter__(self):
        return self._make()

    def map(self, fn):
        return _Dataset(lambda: (fn(*e) if isinstance(e, tuple) and not hasattr(e, "_fields")
                                 else fn(e) for e in self))

    def filter(self, pred):
        return _Dataset(lambda: (e for e in self if pred(*e)))

    def repeat(self, count=None):
        def gen():
            n = 0
            while count is None or count < 0 or n < count:
                empty = True
                for e in self:
                    empty = False
                    yield e
                n += 1
                if empty:
                    return
        return _Dataset(gen)

    def shuffle(self, buffer_size: int, seed: Optional[int] = None):
        def gen():
            rng = np.random.default_rng(seed)
            buf = []
            for e in self:
                if len(buf) < buffer_size:
                    buf.append(e)
                    if len(buf) < buffer_size:
                        continue
                i = int(rng.integers(len(buf)))
                yield buf[i]
                buf[i] = buf[-1]
                buf.pop()
            while buf:
                i = int(rng.integers(len(buf)))
                yield buf[i]
                buf[i] = buf[-1]
                buf.pop()
        return _Dataset(gen)

    def cache(self):
        store: List = []
        done = [False]

        def gen():
            if done[0]:
                yield from store
                return
            store.clear()
            for e in self:
                store.append(e)
                yield e
            done[0] = True
        return _Dataset(gen)

    def prefetch(self, buffer_size: int):
        def gen():
            q: "queue.Queue" = queue.Queue(maxsize=max(1, buffer_size))
            end = object()

            def work():
                try:
                    for e in self:
                        q.put(e)
                    q.put(end)
                except BaseException as ex:          # surfaced in the consumer
                    q.put(ex)
            threading.Thread(target=work, daemon=True).start()
            while True:
                e = q.get()
                if e is end:
                    return
                if isinstance(e, BaseException):
                    raise e
                yield e
        return _Dataset(gen)


def interleave_files(files: Sequence[str], cycle_length: int = 4) -> _Dataset:
    """``parallel_interleave(TFRecordDataset, cycle_length, sloppy=False)`` (block_length 1):
    ``cycle_length`` files are open at once and yield one record each in turn; an exhausted
    file's slot takes the next file."""
    def gen():
        pending = list(files)
        slots: List[Optional[Iterator[bytes]]] = []
        while pending and len(slots) < cycle_length:
            slots.append(R.read_tfrecords(pending.pop(0)))
        while slots:
            i = 0
            while i < len(slots):
                try:
                    yield next(slots[i])
                    i += 1
                except StopIteration:
                    if pending:
                        slots[i] = R.read_tfrecords(pending.pop(0))
                    else:
                        slots.pop(i)
    return _Dataset(gen)


def prepare_target(t: R.PreprocessedMelData, hparams) -> MelData:
    """datasets/ljspeech/dataset.py:126-167."""
    r = hparams.outputs_per_step
    avg = np.asarray(hparams.average_mel_level_db, np.float32)
    std = np.asarray(hparams.stddev_mel_level_db, np.float32)
    sil = np.float32(hparams.silence_mel_level_db)
    mel = (t.mel.astype(np.float32) - avg) / std
    L = int(t.target_length) + 2 * r
    Lp = L if L % r == 0 else (L // r + 1) * r
    out = np.full((Lp, mel.shape[1]), sil, np.float32)
    out[r:r + mel.shape[0]] = mel
    done = np.zeros(Lp // r, np.float32)
    done[-1] = 1.0
    return MelData(t.id, t.key, out, t.mel_width, np.int64(Lp), done,
                   np.ones(Lp, np.float32), np.ones(Lp // r, np.float32))


def prepare_source(s: R.PreprocessedSourceData) -> SourceData:
    return SourceData(s.id, s.key, s.source, s.source_length, s.text)


def _pad_stack(arrays, pad_value, dtype):
    n = max(a.shape[0] for a in arrays)
    out = np.full((len(arrays), n) + arrays[0].shape[1:], pad_value, dtype)
    for i, a in enumerate(arrays):
        out[i, :a.shape[0]] = a
    return out


def padded_batch(elems, hparams):
    """``padded_batch`` with the reference's padded shapes and values (:248-281)."""
    src = [e[0] for e in elems]
    tgt = [e[1] for e in elems]
    sil = hparams.silence_mel_level_db
    s = SourceData(id=np.array([x.id for x in src], np.int64),
                   key=np.array([x.key for x in src], object),
                   source=_pad_stack([x.source for x in src], 0, np.int64),
                   source_length=np.array([x.source_length for x in src], np.int64),
                   text=np.array([x.text for x in src], object))
    t = MelData(id=np.array([x.id for x in tgt], np.int64),
                key=np.array([x.key for x in tgt], object),
                mel=_pad_stack([x.mel for x in tgt], sil, np.float32),
                mel_width=np.array([x.mel_width for x in tgt], np.int64),
                target_length=np.array([x.target_length for x in tgt], np.int64),
                done=_pad_stack([x.done for x in tgt], 1.0, np.float32),
                spec_loss_mask=_pad_stack([x.spec_loss_mask for x in tgt], 0.0, np.float32),
                binary_loss_mask=_pad_stack([x.binary_loss_mask for x in tgt], 0.0, np.float32))
    return s, t


def bucket_key(target_length: int, hparams) -> int:
    """key_func of group_by_batch (:241-244), tf.minimum(.., 0) and floor division included."""
    tl = min(int(target_length) - hparams.approx_min_target_length, 0)
    return min(hparams.batch_num_buckets, tl // hparams.batch_bucket_width)


class DatasetSource:
    """datasets/ljspeech/dataset.py:75-170."""

    def __init__(self, source: Iterable[bytes], target: Iterable[bytes], hparams):
        self._source = source if isinstance(source, _Dataset) else _Dataset(lambda: iter(source))
        self._target = target if isinstance(target, _Dataset) else _Dataset(lambda: iter(target))
        self._hparams = hparams

    @property
    def source(self):
        return self._source

    @property
    def target(self):
        return self._target

    @property
    def hparams(self):
        return self._hparams

    @staticmethod
    def create_from_tfrecord_files(source_files, target_files, hparams, cycle_length=4,
                                   buffer_output_elements=None, prefetch_input_elements=None):
        return DatasetSource(interleave_files(list(source_files), cycle_length),
                             interleave_files(list(target_files), cycle_length), hparams)

    def prepare_and_zip(self) -> "ZippedDataset":
        hp = self.hparams
        src, tgt = self.source, self.target

        def gen():
            for s, t in zip(src, tgt):
                yield (prepare_source(R.parse_preprocessed_source_data(s)),
                       prepare_target(R.parse_preprocessed_mel_data(t), hp))
        return ZippedDataset(_Dataset(gen), hp)


class DatasetBase:
    def apply(self, dataset, hparams):
        raise NotImplementedError("apply")

    @property
    def dataset(self) -> _Dataset:
        raise NotImplementedError("dataset")

    @property
    def hparams(self):
        raise NotImplementedError("hparams")

    def __iter__(self):
        return iter(self.dataset)

    def filter(self, predicate):
        return self.apply(self.dataset.filter(predicate), self.hparams)

    def filter_by_max_output_length(self):
        """Keeps target_length <= max_iters * outputs_per_step (:196-201); the length here is
        the prepared one (silence and rounding included), as in the reference's zipped stream."""
        limit = self.hparams.max_iters * self.hparams.outputs_per_step
        return self.filter(lambda s, t: int(t.target_length) <= limit)

    def shuffle(self, buffer_size, seed=None):
        return self.apply(self.dataset.shuffle(buffer_size, seed), self.hparams)

    def repeat(self, count=None):
        return self.apply(self.dataset.repeat(count), self.hparams)

    def shuffle_and_repeat(self, buffer_size, count=None, seed=None):
        return self.apply(self.dataset.shuffle(buffer_size, seed).repeat(count), self.hparams)

    def cache(self, filename=None):
        """In-memory cache (the reference's file cache name is accepted and unused)."""
        return self.apply(self.dataset.cache(), self.hparams)


class ZippedDataset(DatasetBase):
    def __init__(self, dataset: _Dataset, hparams):
        self._dataset, self._hparams = dataset, hparams

    def apply(self, dataset, hparams):
        return ZippedDataset(dataset, hparams)

    @property
    def dataset(self):
        return self._dataset

    @property
    def hparams(self):
        return self._hparams

    def group_by_batch(self, batch_size=None) -> "BatchedDataset":
        hp = self.hparams
        bs = int(batch_size if batch_size is not None else hp.batch_size)
        window = 5 * bs
        src = self.dataset

        def reduce(elems):
            for i in range(0, len(elems), bs):
                yield padded_batch(elems[i:i + bs], hp)

        def gen():
            windows: "OrderedDict[int, list]" = OrderedDict()
            for e in src:
                k = bucket_key(e[1].target_length, hp)
                w = windows.setdefault(k, [])
                w.append(e)
                if len(w) == window:
                    del windows[k]
                    yield from reduce(w)
            for w in windows.values():
                yield from reduce(w)
        return BatchedDataset(_Dataset(gen), hp)


class BatchedDataset(DatasetBase):
    def __init__(self, dataset: _Dataset, hparams):
        self._dataset, self._hparams = dataset, hparams

    def apply(self, dataset, hparams):
        return BatchedDataset(dataset, self.hparams)

    @property
    def dataset(self):
        return self._dataset

    @property
    def hparams(self):
        return self._hparams

    def prefetch(self, buffer_size):
        return self.apply(self.dataset.prefetch(buffer_size), self.hparams)

    def merge_target_to_source(self):
        """:306-320."""
        def convert(s: SourceData, t: MelData):
            return SourceDataForPrediction(s.id, s.key, s.source, s.source_length, s.text,
                                           t.mel, t.mel_width, t.target_length), t
        return self.apply(self.dataset.map(convert), self.hparams)


def dataset_factory(source, target, hparams):
    """datasets/dataset_factory.py:15-23 with the LJSpeech entry enabled (it is commented out
    in the fork, :12); other names raise ValueError as the reference's factory would."""
    if hparams.dataset in ("ljspeech.dataset.DatasetSource", "datasets.ljspeech.dataset.DatasetSource"):
        return DatasetSource(source, target, hparams)
    raise ValueError(f"Unknown dataset: {hparams.dataset}")


def create_from_tfrecord_files(source_files, target_files, hparams, cycle_length=4,
                               buffer_output_elements=None, prefetch_input_elements=None):
    """datasets/dataset_factory.py:26-32 (LJSpeech entry enabled)."""
    if hparams.dataset in ("ljspeech.dataset.DatasetSource", "datasets.ljspeech.dataset.DatasetSource"):
        return DatasetSource.create_from_tfrecord_files(source_files, target_files, hparams,
                                                        cycle_length, buffer_output_elements,
                                                        prefetch_input_elements)
    raise ValueError(f"Unknown dataset: {hparams.dataset}")


def train_input_fn(hparams, source_files, target_files, seed: Optional[int] = None):
    """train.py:50-56: prepare_and_zip -> filter_by_max_output_length -> repeat ->
    shuffle(suffle_buffer_size) -> group_by_batch -> prefetch."""
    def input_fn():
        ds = create_from_tfrecord_files(source_files, target_files, hparams,
                                        cycle_length=hparams.interleave_cycle_length_min)
        zipped = ds.prepare_and_zip()
        return iter(zipped.filter_by_max_output_length().repeat(count=None)
                    .shuffle(hparams.suffle_buffer_size, seed).group_by_batch()
                    .prefetch(hparams.prefetch_buffer_size))
    return input_fn
