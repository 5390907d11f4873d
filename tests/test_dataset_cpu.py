"""Dataset path without a GPU: TFRecord framing + CRC-32C in libsat_hip's
host entries, the tf.train.Example wire format, and the LJSpeech pipeline contract of
datasets/ljspeech/dataset.py:126-167, 237-285 (prepare, bucket, pad).

Pinning: CRC-32C against its published check value (RFC 3720 B.4 "123456789" -> 0xE3069283 and
the 32-zero-byte vector); the Example codec against message classes the protobuf library builds
from the tf.train.Example .proto definitions (example.proto / feature.proto field numbers,
restated here as a descriptor -- TensorFlow itself is not installed); the pipeline against the
reference's formulas evaluated by hand on small inputs."""
import os

import numpy as np
import pytest

import _sat_path

_sat_path.load()
from sat_amd import datasets as D  # noqa: E402
from sat_amd import hparams  # noqa: E402
from sat_amd import tfrecord as R  # noqa: E402


# ---------------------------------------------------------------- framing
def test_crc32c_known_answers():
    from sat_amd import _lib
    L = _lib.load()
    assert L.sat_crc32c(b"123456789", 9, 0) == 0xE3069283
    assert L.sat_crc32c(bytes(32), 32, 0) == 0x8A9136AA
    assert L.sat_crc32c(b"\xff" * 32, 32, 0) == 0x62A8AB43
    data = os.urandom(1001)                                        # continuation == one pass
    assert L.sat_crc32c(data[500:], 501, L.sat_crc32c(data[:500], 500, 0)) == \
        L.sat_crc32c(data, 1001, 0)
    c = L.sat_crc32c(b"abc", 3, 0)
    assert L.sat_tfrecord_masked_crc(b"abc", 3) == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF)
                                                    + 0xA282EAD8) & 0xFFFFFFFF


def test_record_framing_round_trip_and_corruption(tmp_path):
    recs = [b"", b"x", os.urandom(70000)]
    f = str(tmp_path / "a.tfrecord")
    R.write_tfrecords(recs, f)
    raw = open(f, "rb").read()
    assert len(raw) == sum(len(r) + 16 for r in recs)
    assert int.from_bytes(raw[:8], "little") == 0
    assert list(R.read_tfrecords(f)) == recs
    bad = bytearray(raw)
    bad[60] ^= 1                                                   # inside record 2's payload
    with pytest.raises(ValueError, match="checksum"):
        R.split_records(bytes(bad))
    assert len(R.split_records(bytes(bad), verify=False)) == 3
    with pytest.raises(ValueError, match="truncated"):
        R.split_records(raw[:-3])


# ---------------------------------------------------------------- tf.train.Example
def _example_classes():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name="sat_example_test.proto",
                                            package="sat_test", syntax="proto3")
    T = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields, nested=()):
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
        for n in nested:
            m.nested_type.add().CopyFrom(n)
        return m

    rep, opt = T.LABEL_REPEATED, T.LABEL_OPTIONAL
    msg("BytesList", [("value", 1, T.TYPE_BYTES, rep, None)])
    msg("FloatList", [("value", 1, T.TYPE_FLOAT, rep, None)])
    msg("Int64List", [("value", 1, T.TYPE_INT64, rep, None)])
    msg("Feature", [("bytes_list", 1, T.TYPE_MESSAGE, opt, ".sat_test.BytesList"),
                    ("float_list", 2, T.TYPE_MESSAGE, opt, ".sat_test.FloatList"),
                    ("int64_list", 3, T.TYPE_MESSAGE, opt, ".sat_test.Int64List")])
    entry = descriptor_pb2.DescriptorProto(name="FeatureEntry")
    entry.field.add(name="key", number=1, type=T.TYPE_STRING, label=opt)
    entry.field.add(name="value", number=2, type=T.TYPE_MESSAGE, label=opt,
                    type_name=".sat_test.Feature")
    entry.options.map_entry = True
    msg("Features", [("feature", 1, T.TYPE_MESSAGE, rep, ".sat_test.Features.FeatureEntry")],
        nested=[entry])
    msg("Example", [("features", 1, T.TYPE_MESSAGE, opt, ".sat_test.Features")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = getattr(message_factory, "GetMessageClass", None)
    return {n: get(pool.FindMessageTypeByName(f"sat_test.{n}")) for n in
            ("Example", "Feature", "BytesList", "FloatList", "Int64List")}


def test_example_codec_matches_protobuf():
    C = _example_classes()
    feats = {"id": ("int64", [7]), "neg": ("int64", [-3, 0, 1 << 40]),
             "key": ("bytes", [b"LJ001-0001"]), "f": ("float", [1.5, -2.25]),
             "empty": ("int64", [])}
    ours = R.encode_example(feats)
    ex = C["Example"]()
    ex.ParseFromString(ours)                                    # protobuf reads our bytes
    fm = ex.features.feature
    assert list(fm["id"].int64_list.value) == [7]
    assert list(fm["neg"].int64_list.value) == [-3, 0, 1 << 40]
    assert list(fm["key"].bytes_list.value) == [b"LJ001-0001"]
    assert list(fm["f"].float_list.value) == [1.5, -2.25]
    # and we read protobuf's bytes (its own map ordering / packing)
    assert R.decode_example(ex.SerializeToString()) == feats
    # unpacked numeric lists (proto2-style writers) decode too
    unpacked = bytes([0x0A, 0x0F, 0x0A, 0x0D, 0x0A, 0x01]) + b"a" + bytes(
        [0x12, 0x08, 0x1A, 0x06, 0x08, 0x05, 0x08, 0x7F, 0x08, 0x01])
    assert R.decode_example(unpacked) == {"a": ("int64", [5, 127, 1])}


def test_ljspeech_record_types_round_trip(tmp_path):
    src = np.array([5, 12, 70, 1], np.int64)
    mel = np.random.default_rng(0).standard_normal((9, 80)).astype(np.float32)
    R.write_preprocessed_source_data(3, "LJ-3", src, "text!", str(tmp_path / "s"))
    R.write_preprocessed_target_data(3, "LJ-3", mel, str(tmp_path / "t"))
    s = R.parse_preprocessed_source_data(next(R.read_tfrecords(str(tmp_path / "s"))))
    t = R.parse_preprocessed_mel_data(next(R.read_tfrecords(str(tmp_path / "t"))))
    assert (s.id, s.key, s.source_length, s.text) == (3, b"LJ-3", 4, b"text!")
    np.testing.assert_array_equal(s.source, src)
    assert (t.id, t.target_length, t.mel_width) == (3, 9, 80)
    np.testing.assert_array_equal(t.mel, mel)
    with pytest.raises(ValueError, match="required"):
        R.parse_preprocessed_mel_data(R.encode_example({"id": ("int64", [1])}))


# ---------------------------------------------------------------- pipeline contract
def _hp(**kw):
    hp = hparams.ljspeech_hparams()
    hp.set_hparam("average_mel_level_db", [1.0] * 80)
    hp.set_hparam("stddev_mel_level_db", [2.0] * 80)
    for k, v in kw.items():
        hp.set_hparam(k, v)
    return hp


def test_prepare_target_contract():
    hp = _hp()
    r, sil = hp.outputs_per_step, hp.silence_mel_level_db
    for T in (5, 6):
        mel = np.full((T, 80), 5.0, np.float32)
        t = D.prepare_target(R.PreprocessedMelData(1, b"k", mel, T, 80), hp)
        L = T + 2 * r
        Lp = L if L % r == 0 else (L // r + 1) * r                   # dataset.py:141-154
        assert t.target_length == Lp and t.mel.shape == (Lp, 80)
        np.testing.assert_array_equal(t.mel[:r], sil)
        np.testing.assert_array_equal(t.mel[r:r + T], 2.0)           # (5 - 1) / 2
        np.testing.assert_array_equal(t.mel[r + T:], sil)
        np.testing.assert_array_equal(t.done, [0.0] * (Lp // r - 1) + [1.0])
        np.testing.assert_array_equal(t.spec_loss_mask, 1.0)
        assert t.binary_loss_mask.shape == (Lp // r,)


def test_bucket_key_keeps_reference_minimum():
    hp = _hp()
    assert D.bucket_key(100, hp) == D.bucket_key(990, hp) == 0      # tf.minimum(len - 100, 0)
    assert D.bucket_key(99, hp) == -1 and D.bucket_key(50, hp) == -1
    assert D.bucket_key(49, hp) == -2                                # floor division


def _write_corpus(tmp_path, lengths, n_chars, files_per=1):
    rng = np.random.default_rng(1)
    srcs, tgts = [], []
    for i, (T, N) in enumerate(zip(lengths, n_chars)):
        s, t = str(tmp_path / f"{i}.source.tfrecord"), str(tmp_path / f"{i}.target.tfrecord")
        R.write_preprocessed_source_data(i, f"LJ{i:03d}", rng.integers(1, 71, N), f"t{i}", s)
        R.write_preprocessed_target_data(i, f"LJ{i:03d}",
                                         rng.standard_normal((T, 80)).astype(np.float32), t)
        srcs.append(s)
        tgts.append(t)
    return srcs, tgts


def test_pipeline_batches_and_padding(tmp_path):
    hp = _hp(max_iters=60)
    lengths = [110, 90, 40, 101, 95, 30, 200, 118]
    chars = [20, 15, 9, 30, 12, 7, 40, 25]
    srcs, tgts = _write_corpus(tmp_path, lengths, chars)
    ds = D.DatasetSource.create_from_tfrecord_files(srcs, tgts, hp, cycle_length=3)
    zipped = ds.prepare_and_zip()
    ids = [int(s.id) for s, _ in zipped]
    # parallel_interleave(cycle 3, sloppy=False): one record per open file, in turn
    assert ids == list(range(8))
    batches = list(zipped.filter_by_max_output_length().group_by_batch(batch_size=2))
    seen = sorted(int(i) for s, _ in batches for i in s.id)
    assert seen == [i for i in range(8) if lengths[i] + 2 * 2 <= 120]   # 200-frame one dropped
    sil = hp.silence_mel_level_db
    for s, t in batches:
        B = len(s.id)
        assert B <= 2
        n_max, t_max = s.source.shape[1], t.mel.shape[1]
        assert n_max == s.source_length.max() and t_max == t.target_length.max()
        for b in range(B):
            n, T = int(s.source_length[b]), int(t.target_length[b])
            assert (s.source[b, n:] == 0).all()
            assert (t.mel[b, T:] == sil).all()
            assert (t.spec_loss_mask[b, :T] == 1).all() and (t.spec_loss_mask[b, T:] == 0).all()
            assert (t.binary_loss_mask[b, :T // 2] == 1).all()
            assert (t.binary_loss_mask[b, T // 2:] == 0).all()
            assert (t.done[b, T // 2 - 1:] == 1).all() and (t.done[b, :T // 2 - 1] == 0).all()
    # buckets: all >= 100-frame utterances share key 0; 40/30-frame ones key -2 / -2, 90/95 -1
    keys = [[D.bucket_key(int(x), hp) for x in t.target_length] for _, t in batches]
    assert all(len(set(k)) == 1 for k in keys)


def test_group_by_window_emits_full_windows_first(tmp_path):
    """A window of 5*batch_size same-key elements is emitted as soon as it fills; partial
    windows are flushed at the end, in order of first appearance (group_by_window)."""
    hp = _hp(max_iters=500)
    lengths = [50] + [120] * 10 + [60]
    srcs, tgts = _write_corpus(tmp_path, lengths, [5] * 12)
    batches = list(D.DatasetSource.create_from_tfrecord_files(srcs, tgts, hp, cycle_length=1)
                   .prepare_and_zip().group_by_batch(batch_size=2))
    order = [list(map(int, s.id)) for s, _ in batches]
    assert order[:5] == [[1, 2], [3, 4], [5, 6], [7, 8], [9, 10]]     # key-0 window of 10
    assert order[5:] == [[0, 11]]                                     # key -1, flushed
    assert sorted(i for b in order for i in b) == list(range(12))


def test_train_input_fn_feeds_model_fn_records(tmp_path):
    hp = _hp(max_iters=80, batch_size=2)
    srcs, tgts = _write_corpus(tmp_path, [100, 110, 120, 130], [10, 11, 12, 13])
    it = D.train_input_fn(hp, srcs, tgts, seed=0)()
    s, t = next(it)
    assert s.source.dtype == np.int64 and t.mel.dtype == np.float32
    assert t.mel.shape[0] == 2 and t.mel.shape[2] == 80 and t.mel.shape[1] % 2 == 0
    assert hasattr(t, "spec_loss_mask") and hasattr(t, "binary_loss_mask")


def test_dataset_factory_names():
    hp = _hp()
    assert isinstance(D.dataset_factory([], [], hp), D.DatasetSource)
    hp.set_hparam("dataset", "codes.dataset.DatasetSource")
    with pytest.raises(ValueError, match="Unknown dataset"):
        D.dataset_factory([], [], hp)


def test_shuffle_repeat_merge(tmp_path):
    """shuffle (buffer algorithm of tf.data: a permutation, seeded), repeat(count), cache and
    merge_target_to_source (:306-320: SourceDataForPrediction carries the target mel)."""
    hp = _hp(max_iters=500)
    srcs, tgts = _write_corpus(tmp_path, [120, 130, 140, 150, 160], [5, 6, 7, 8, 9])
    z = D.DatasetSource.create_from_tfrecord_files(srcs, tgts, hp, cycle_length=2).prepare_and_zip()
    ids = [int(s.id) for s, _ in z]
    assert sorted(ids) == list(range(5))
    sh = [int(s.id) for s, _ in z.shuffle(3, seed=1)]
    assert sorted(sh) == sorted(ids)
    assert sh == [int(s.id) for s, _ in z.shuffle(3, seed=1)]           # seeded: repeatable
    assert [int(s.id) for s, _ in z.repeat(2)] == ids + ids
    c = z.cache()
    assert [int(s.id) for s, _ in c] == [int(s.id) for s, _ in c] == ids
    s, t = next(iter(z.group_by_batch(batch_size=5).merge_target_to_source()))
    assert isinstance(s, D.SourceDataForPrediction)
    np.testing.assert_array_equal(s.mel, t.mel)
    np.testing.assert_array_equal(s.target_length, t.target_length)
