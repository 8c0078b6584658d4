"""Native DICOM reader (innovative3D/dicom.py), the pydicom-less path of
read_dicom_frames (reference helpers.py:190-191: ``pydicom.dcmread(fn).pixel_array``).

Parity with pydicom is unpinned (pydicom is absent offline, and no DICOM file ships with
the reference): the expected arrays follow pydicom's documented pixel_array semantics, and
the inputs are (a) a byte stream assembled by hand in this file, tag by tag, and (b) files
from the small Part-10 writer below, in every supported transfer syntax."""
import struct
import zlib

import numpy as np
import pytest

from innovative3D import dicom as D
from innovative3D.helpers import read_dicom_frames

_LONG = {"OB", "OD", "OF", "OL", "OV", "OW", "SQ", "UC", "UN", "UR", "UT"}


def _el(g, e, vr, val, explicit=True):
    if isinstance(val, str):
        val = val.encode("ascii")
        if len(val) % 2:
            val += b"\x00" if vr == "UI" else b" "
    if not explicit:
        return struct.pack("<HHI", g, e, len(val)) + val
    if vr in _LONG:
        return struct.pack("<HH2sHI", g, e, vr.encode(), 0, len(val)) + val
    return struct.pack("<HH2sH", g, e, vr.encode(), len(val)) + val


def _us(v):
    return struct.pack("<H", v)


def _sq_undefined(explicit):
    """A sequence of undefined length holding one undefined-length item with a nested
    defined-length sequence -- the reader must skip it by its delimiters."""
    inner = _el(0x0008, 0x0100, "SH", "CODE1", explicit)
    nested = _el(0x0008, 0x0104, "LO", "meaning", explicit)
    nested_sq = (_el(0x0040, 0xA043, "SQ", struct.pack("<HHI", 0xFFFE, 0xE000, len(nested)) + nested,
                     explicit))
    item = (struct.pack("<HHI", 0xFFFE, 0xE000, 0xFFFFFFFF) + inner + nested_sq +
            struct.pack("<HHI", 0xFFFE, 0xE00D, 0))
    if explicit:
        head = struct.pack("<HH2sHI", 0x0008, 0x1140, b"SQ", 0, 0xFFFFFFFF)
    else:
        head = struct.pack("<HHI", 0x0008, 0x1140, 0xFFFFFFFF)
    return head + item + struct.pack("<HHI", 0xFFFE, 0xE0DD, 0)


def write_dicom(frames, ts=D.EXPLICIT_LE, bits_stored=None, signed=None, planar=0,
                preamble=True, with_sq=True):
    """Minimal Part-10 writer: frames [F, R, C] or [F, R, C, S] integer array."""
    a = np.asarray(frames)
    if a.ndim == 2:
        a = a[None]
    spp = a.shape[3] if a.ndim == 4 else 1
    F, R, C = a.shape[:3]
    ba = a.dtype.itemsize * 8
    signed = a.dtype.kind == "i" if signed is None else signed
    explicit = ts != D.IMPLICIT_LE
    body = b""
    if with_sq:
        body += _sq_undefined(explicit)
    body += _el(0x0010, 0x0010, "PN", "Anon^Phantom", explicit)
    body += _el(0x0028, 0x0002, "US", _us(spp), explicit)
    body += _el(0x0028, 0x0004, "CS", "MONOCHROME2" if spp == 1 else "RGB", explicit)
    if spp > 1:
        body += _el(0x0028, 0x0006, "US", _us(planar), explicit)
    body += _el(0x0028, 0x0008, "IS", str(F), explicit)
    body += _el(0x0028, 0x0010, "US", _us(R), explicit)
    body += _el(0x0028, 0x0011, "US", _us(C), explicit)
    body += _el(0x0028, 0x0100, "US", _us(ba), explicit)
    body += _el(0x0028, 0x0101, "US", _us(bits_stored or ba), explicit)
    body += _el(0x0028, 0x0103, "US", _us(1 if signed else 0), explicit)
    pix = a.transpose(0, 3, 1, 2) if (spp > 1 and planar == 1) else a
    raw = np.ascontiguousarray(pix).astype(a.dtype.newbyteorder("<")).tobytes()
    if len(raw) % 2:
        raw += b"\x00"
    body += _el(0x7FE0, 0x0010, "OW" if ba > 8 else "OB", raw, explicit)
    if ts == D.DEFLATED_LE:
        co = zlib.compressobj(9, zlib.DEFLATED, -15)
        body = co.compress(body) + co.flush()
    if not preamble:
        return body
    meta = _el(0x0002, 0x0010, "UI", ts)
    meta = _el(0x0002, 0x0000, "UL", struct.pack("<I", len(meta))) + meta
    return b"\x00" * 128 + b"DICM" + meta + body


def test_hand_assembled_stream():
    # explicit VR little endian, 2 frames of 2 x 3 uint16, bytes laid out by hand
    meta_ts = b"1.2.840.10008.1.2.1\x00"
    meta = struct.pack("<HH2sH", 2, 0x10, b"UI", len(meta_ts)) + meta_ts
    ds = b"".join([
        struct.pack("<HH2sH", 0x28, 0x02, b"US", 2) + struct.pack("<H", 1),
        struct.pack("<HH2sH", 0x28, 0x08, b"IS", 2) + b"2 ",
        struct.pack("<HH2sH", 0x28, 0x10, b"US", 2) + struct.pack("<H", 2),
        struct.pack("<HH2sH", 0x28, 0x11, b"US", 2) + struct.pack("<H", 3),
        struct.pack("<HH2sH", 0x28, 0x100, b"US", 2) + struct.pack("<H", 16),
        struct.pack("<HH2sH", 0x28, 0x101, b"US", 2) + struct.pack("<H", 16),
        struct.pack("<HH2sH", 0x28, 0x103, b"US", 2) + struct.pack("<H", 0),
        struct.pack("<HH2sHI", 0x7FE0, 0x10, b"OW", 0, 24) + struct.pack("<12H", *range(100, 112)),
    ])
    buf = b"\x00" * 128 + b"DICM" + meta + ds
    a = D.pixel_array(buf)
    assert a.dtype == np.uint16 and a.shape == (2, 2, 3)
    np.testing.assert_array_equal(a, np.arange(100, 112, dtype=np.uint16).reshape(2, 2, 3))


@pytest.mark.parametrize("ts", [D.EXPLICIT_LE, D.IMPLICIT_LE, D.DEFLATED_LE])
@pytest.mark.parametrize("dtype", [np.uint8, np.int8, np.uint16, np.int16, np.uint32, np.int32])
def test_round_trip(ts, dtype, tmp_path):
    rng = np.random.default_rng(7)
    info = np.iinfo(dtype)
    a = rng.integers(info.min, info.max, size=(5, 12, 10), dtype=dtype, endpoint=True)
    p = tmp_path / "x.dcm"
    p.write_bytes(write_dicom(a, ts))
    got = D.pixel_array(str(p))
    assert got.dtype == np.dtype(dtype) and got.shape == a.shape
    np.testing.assert_array_equal(got, a)
    np.testing.assert_array_equal(read_dicom_frames(str(p)), a)  # the data path's reader


def test_single_frame_drops_the_frame_axis():
    a = np.arange(6 * 4, dtype=np.uint16).reshape(1, 6, 4)
    got = D.pixel_array(write_dicom(a))
    assert got.shape == (6, 4)  # pydicom: (rows, cols) for one frame
    np.testing.assert_array_equal(got, a[0])


def test_signed_bits_stored_sign_extends():
    # 12-bit signed values stored in 16 bits with garbage-free high bits: -5 -> 0x0FFB
    vals = np.array([[[-5, 7], [-2048, 2047]]], dtype=np.int16)
    stored = (vals.astype(np.int32) & 0x0FFF).astype(np.uint16).view(np.int16)
    got = D.pixel_array(write_dicom(np.concatenate([stored, stored]), bits_stored=12,
                                    signed=True))
    np.testing.assert_array_equal(got, np.concatenate([vals, vals]))


@pytest.mark.parametrize("planar", [0, 1])
def test_rgb_samples(planar):
    a = np.arange(2 * 3 * 4 * 3, dtype=np.uint8).reshape(2, 3, 4, 3)
    got = D.pixel_array(write_dicom(a, planar=planar))
    assert got.shape == (2, 3, 4, 3)
    np.testing.assert_array_equal(got, a)


def test_bare_dataset_without_preamble():
    a = np.arange(3 * 5 * 7, dtype=np.int16).reshape(3, 5, 7) - 50
    got = D.pixel_array(write_dicom(a, D.IMPLICIT_LE, preamble=False, with_sq=False))
    np.testing.assert_array_equal(got, a)


def test_compressed_and_broken_inputs_fail_loudly():
    jpeg = write_dicom(np.zeros((2, 4, 4), np.uint8), "1.2.840.10008.1.2.4.50")
    with pytest.raises(NotImplementedError):
        D.pixel_array(jpeg)
    # encapsulated pixel data in a JPEG transfer syntax: well-formed items, no codec
    jpeg_encap = write_rle_dicom(np.zeros((1, 4, 4), np.uint8), ts="1.2.840.10008.1.2.4.70")
    with pytest.raises(NotImplementedError):
        D.pixel_array(jpeg_encap)
    encap = bytearray(write_dicom(np.zeros((1, 4, 4), np.uint8), with_sq=False))
    i = encap.index(struct.pack("<HH", 0x7FE0, 0x10))
    encap[i + 8:i + 12] = struct.pack("<I", 0xFFFFFFFF)  # undefined length, no items
    with pytest.raises(D.DicomError):
        D.pixel_array(bytes(encap))
    good = write_dicom(np.zeros((2, 4, 4), np.uint16))
    with pytest.raises(D.DicomError):
        D.pixel_array(good[:-9])


# ---- RLE Lossless (PS3.5 Annex G), encoded here independently of the reader ----
def _packbits(data: bytes) -> bytes:
    """PackBits as PS3.5 G.3.1 describes it: replicate runs of 3 .. 128 bytes as
    (257 - n, byte), literal runs of 1 .. 128 bytes as (n - 1, bytes...)"""
    out, i, n = bytearray(), 0, len(data)
    while i < n:
        j = i
        while j + 1 < n and data[j + 1] == data[i] and j + 1 - i < 127:
            j += 1
        run = j - i + 1
        if run >= 3:
            out += bytes((257 - run, data[i]))
            i = j + 1
            continue
        k = i
        while k < n and k - i < 128:
            if k + 2 < n and data[k] == data[k + 1] == data[k + 2]:
                break
            k += 1
        out += bytes((k - i - 1,)) + data[i:k]
        i = k
    if len(out) % 2:
        out += bytes((128,))  # a no-op pad byte keeps the segment even
    return bytes(out)


def _rle_frame(frame: np.ndarray) -> bytes:
    """[R, C] or [R, C, S] -> one RLE frame: header + segments per sample, MSB first"""
    f = frame if frame.ndim == 3 else frame[..., None]
    nb = f.dtype.itemsize
    segs = []
    u = f.astype(f.dtype.newbyteorder("<")).view(np.uint8).reshape(f.shape[0] * f.shape[1],
                                                                     f.shape[2], nb)
    for smp in range(f.shape[2]):
        for k in range(nb):
            segs.append(_packbits(np.ascontiguousarray(u[:, smp, nb - 1 - k]).tobytes()))
    offs, o = [], 64
    for sg in segs:
        offs.append(o)
        o += len(sg)
    head = struct.pack("<I", len(segs)) + struct.pack("<15I", *(offs + [0] * (15 - len(offs))))
    return head + b"".join(segs)


def write_rle_dicom(frames, ts=D.RLE_LOSSLESS, signed=None):
    a = np.asarray(frames)
    spp = a.shape[3] if a.ndim == 4 else 1
    F, R, C = a.shape[:3]
    ba = a.dtype.itemsize * 8
    signed = a.dtype.kind == "i" if signed is None else signed
    body = _sq_undefined(True)
    body += _el(0x0028, 0x0002, "US", _us(spp))
    body += _el(0x0028, 0x0004, "CS", "MONOCHROME2" if spp == 1 else "RGB")
    if spp > 1:
        body += _el(0x0028, 0x0006, "US", _us(1))  # RLE images are by plane (PS3.5 G.2)
    body += _el(0x0028, 0x0008, "IS", str(F))
    body += _el(0x0028, 0x0010, "US", _us(R))
    body += _el(0x0028, 0x0011, "US", _us(C))
    body += _el(0x0028, 0x0100, "US", _us(ba))
    body += _el(0x0028, 0x0101, "US", _us(ba))
    body += _el(0x0028, 0x0103, "US", _us(1 if signed else 0))
    items = struct.pack("<HHI", 0xFFFE, 0xE000, 0)  # empty Basic Offset Table
    for f in range(F):
        fr = _rle_frame(a[f])
        items += struct.pack("<HHI", 0xFFFE, 0xE000, len(fr)) + fr
    body += struct.pack("<HH2sHI", 0x7FE0, 0x10, b"OB", 0, 0xFFFFFFFF) + items
    body += struct.pack("<HHI", 0xFFFE, 0xE0DD, 0)
    meta = _el(0x0002, 0x0010, "UI", ts)
    meta = _el(0x0002, 0x0000, "UL", struct.pack("<I", len(meta))) + meta
    return b"\x00" * 128 + b"DICM" + meta + body


@pytest.mark.parametrize("dtype", [np.uint8, np.int8, np.uint16, np.int16, np.int32])
def test_rle_lossless_round_trip(dtype):
    rng = np.random.default_rng(3)
    info = np.iinfo(dtype)
    a = rng.integers(info.min, info.max, size=(3, 9, 14), dtype=dtype, endpoint=True)
    a[:, 2:6, 3:11] = a[0, 0, 0]  # long replicate runs beside literal ones
    got = D.pixel_array(write_rle_dicom(a))
    assert got.dtype == np.dtype(dtype) and got.shape == a.shape
    np.testing.assert_array_equal(got, a)
    one = D.pixel_array(write_rle_dicom(a[:1]))
    np.testing.assert_array_equal(one, a[0])  # one frame: (rows, cols)


def test_rle_lossless_rgb_and_packbits_edge_cases():
    a = np.zeros((2, 5, 40, 3), np.uint8)
    a[0, :, :, 1] = 7                      # a 200-byte run: split into runs of <= 128
    a[1] = np.arange(600, dtype=np.uint8).reshape(5, 40, 3)  # literal runs > 128
    got = D.pixel_array(write_rle_dicom(a))
    assert got.shape == a.shape
    np.testing.assert_array_equal(got, a)
    assert D._unpackbits(bytes((254, 9, 128, 1, 5, 6)), 5) == bytes((9, 9, 9, 5, 6))
