"""Native DICOM Part-10 reader for uncompressed pixel data (numpy only).

The reference decodes each DICOM stack with ``pydicom.dcmread(path).pixel_array``
(helpers.py:190-191).  pydicom is not installed here, so this module restates the part of
the standard that path needs (PS3.5 data-element encoding, PS3.10 file format):

* the 128-byte preamble + ``DICM`` (or a bare dataset, read as implicit VR little endian),
* the file meta group (always explicit VR little endian) and its Transfer Syntax UID,
* Implicit VR Little Endian (1.2.840.10008.1.2), Explicit VR Little Endian
  (1.2.840.10008.1.2.1) and Deflated Explicit VR Little Endian (1.2.840.10008.1.2.1.99),
* elements of undefined length (sequences, items) skipped by their delimiters,
* native pixel data -> the array ``pixel_array`` would return: dtype from Bits Allocated and
  Pixel Representation (signed values sign-extended from Bits Stored), shape
  (frames, rows, cols[, samples]) with the frame axis dropped for a single frame, planar
  configuration 1 reordered to interleaved samples.

* RLE Lossless (1.2.840.10008.1.2.5, PS3.5 Annex G): the encapsulated fragments (one per
  frame, after the Basic Offset Table item) decoded as pydicom's built-in RLE handler does:
  per frame up to 15 PackBits segments, one per sample and byte (most significant first).

Other encapsulated (compressed) transfer syntaxes -- JPEG, JPEG-LS, JPEG 2000 -- need an
image codec (pydicom itself decodes them only with a plugin such as pylibjpeg or GDCM
installed) and raise ``NotImplementedError``.  Parity with pydicom is unpinned (pydicom is
absent and no DICOM files are available offline); the tests check hand-assembled byte
streams and round trips through an independent writer / RLE encoder.
"""
from __future__ import annotations

import struct
import zlib
from typing import Dict, Tuple

import numpy as np

IMPLICIT_LE = "1.2.840.10008.1.2"
EXPLICIT_LE = "1.2.840.10008.1.2.1"
DEFLATED_LE = "1.2.840.10008.1.2.1.99"
EXPLICIT_BE = "1.2.840.10008.1.2.2"
RLE_LOSSLESS = "1.2.840.10008.1.2.5"

# explicit VRs with a 2-byte reserved field and a 4-byte length (PS3.5 7.1.2)
_LONG_VRS = {b"OB", b"OD", b"OF", b"OL", b"OV", b"OW", b"SQ", b"UC", b"UN", b"UR", b"UT", b"SV",
             b"UV"}
_UNDEFINED = 0xFFFFFFFF
_ITEM, _ITEM_END, _SEQ_END = (0xFFFE, 0xE000), (0xFFFE, 0xE00D), (0xFFFE, 0xE0DD)

# the image attributes pixel decoding needs: (group, element) -> keyword
_WANTED = {
    (0x0028, 0x0002): "SamplesPerPixel",
    (0x0028, 0x0004): "PhotometricInterpretation",
    (0x0028, 0x0006): "PlanarConfiguration",
    (0x0028, 0x0008): "NumberOfFrames",
    (0x0028, 0x0010): "Rows",
    (0x0028, 0x0011): "Columns",
    (0x0028, 0x0100): "BitsAllocated",
    (0x0028, 0x0101): "BitsStored",
    (0x0028, 0x0103): "PixelRepresentation",
    (0x7FE0, 0x0010): "PixelData",
}
_US = {"SamplesPerPixel", "PlanarConfiguration", "Rows", "Columns", "BitsAllocated",
       "BitsStored", "PixelRepresentation"}


class DicomError(ValueError):
    pass


def _header(buf: bytes, pos: int, explicit: bool) -> Tuple[Tuple[int, int], bytes, int, int]:
    """(tag, VR or b'', value length, value offset) of the element at pos."""
    if pos + 8 > len(buf):
        raise DicomError(f"truncated element header at byte {pos}")
    g, e = struct.unpack_from("<HH", buf, pos)
    if (g, e) in (_ITEM, _ITEM_END, _SEQ_END):  # item / delimiters: always tag + u32 length
        (n,) = struct.unpack_from("<I", buf, pos + 4)
        return (g, e), b"", n, pos + 8
    if not explicit:
        (n,) = struct.unpack_from("<I", buf, pos + 4)
        return (g, e), b"", n, pos + 8
    vr = buf[pos + 4:pos + 6]
    if vr in _LONG_VRS:
        if pos + 12 > len(buf):
            raise DicomError(f"truncated element header at byte {pos}")
        (n,) = struct.unpack_from("<I", buf, pos + 8)
        return (g, e), vr, n, pos + 12
    (n,) = struct.unpack_from("<H", buf, pos + 6)
    return (g, e), vr, n, pos + 8


def _skip_undefined(buf: bytes, pos: int, explicit: bool) -> int:
    """pos = first byte after an undefined-length element's header; returns the offset after
    its Sequence Delimitation Item (items of defined or undefined length, nested)."""
    while True:
        tag, _vr, n, v = _header(buf, pos, explicit)
        if tag == _SEQ_END:
            return v
        if tag != _ITEM:
            raise DicomError(f"expected an item in an undefined-length sequence at byte {pos}")
        if n != _UNDEFINED:
            pos = v + n
            continue
        pos = v  # undefined-length item: its elements up to the Item Delimitation Item
        while True:
            tag, _vr, n, v = _header(buf, pos, explicit)
            if tag == _ITEM_END:
                pos = v
                break
            pos = _skip_undefined(buf, v, explicit) if n == _UNDEFINED else v + n


def _fragments(buf: bytes, pos: int, explicit: bool) -> Tuple[list, int]:
    """Encapsulated pixel data (PS3.5 A.4): the items after the element header at pos, up to
    the Sequence Delimitation Item -> ([Basic Offset Table, fragment, ...], end offset)."""
    items = []
    while True:
        tag, _vr, n, v = _header(buf, pos, explicit)
        if tag == _SEQ_END:
            return items, v
        if tag != _ITEM or n == _UNDEFINED or v + n > len(buf):
            raise DicomError(f"malformed encapsulated pixel data item at byte {pos}")
        items.append(buf[v:v + n])
        pos = v + n


def _parse(buf: bytes, pos: int, explicit: bool, stop_group: int = None,
           out: Dict = None) -> Tuple[Dict, int]:
    """Top-level elements from pos: keeps _WANTED values (raw bytes) and (0002,0010);
    encapsulated pixel data as the list of its items."""
    out = {} if out is None else out
    while pos < len(buf):
        if stop_group is not None:
            (g,) = struct.unpack_from("<H", buf, pos)
            if g != stop_group:
                break
        tag, vr, n, v = _header(buf, pos, explicit)
        if n == _UNDEFINED:
            if tag == (0x7FE0, 0x0010):
                out[tag], pos = _fragments(buf, v, explicit)
                continue
            pos = _skip_undefined(buf, v, explicit)
            continue
        if v + n > len(buf):
            raise DicomError(f"element {tag[0]:04X},{tag[1]:04X} runs past the end of the file")
        if tag in _WANTED or tag == (0x0002, 0x0010):
            out[tag] = (vr, buf[v:v + n])
        pos = v + n
    return out, pos


def _text(raw: bytes) -> str:
    return raw.decode("ascii", "replace").strip("\x00 ").strip()


def read_dataset(path_or_bytes) -> Dict[str, object]:
    """The image attributes of one DICOM file (keywords as in the standard) plus
    ``TransferSyntaxUID``; PixelData stays raw bytes."""
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
        buf = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as f:
            buf = f.read()
    ts = IMPLICIT_LE
    if len(buf) >= 132 and buf[128:132] == b"DICM":
        meta, pos = _parse(buf, 132, True, stop_group=0x0002)
        if (0x0002, 0x0010) in meta:
            ts = _text(meta[(0x0002, 0x0010)][1])
    else:  # no preamble: a bare dataset in the default transfer syntax
        pos = 0
    if ts == DEFLATED_LE:
        buf, pos = zlib.decompress(buf[pos:], -15), 0
        explicit = True
    elif ts in (IMPLICIT_LE, EXPLICIT_LE, RLE_LOSSLESS):
        explicit = ts != IMPLICIT_LE
    elif ts == EXPLICIT_BE:
        raise NotImplementedError("Explicit VR Big Endian (retired) is not supported")
    else:
        raise NotImplementedError(f"transfer syntax {ts}: compressed pixel data needs a codec")
    raw, _ = _parse(buf, pos, explicit)
    ds: Dict[str, object] = {"TransferSyntaxUID": ts}
    for tag, item in raw.items():
        key = _WANTED.get(tag)
        if key is None:
            continue
        if key == "PixelData" and isinstance(item, list):
            ds[key] = item  # encapsulated: [Basic Offset Table, fragment, ...]
            continue
        vr, val = item
        if key in _US:
            if len(val) < 2:
                raise DicomError(f"{key}: empty value")
            ds[key] = struct.unpack_from("<H", val)[0]
        elif key == "NumberOfFrames":
            ds[key] = int(_text(val) or "1")
        elif key == "PhotometricInterpretation":
            ds[key] = _text(val)
        else:
            ds[key] = val
    return ds


def pixel_array(path_or_bytes) -> np.ndarray:
    """``pydicom.dcmread(path).pixel_array`` for native (uncompressed) pixel data."""
    ds = read_dataset(path_or_bytes)
    for k in ("Rows", "Columns", "BitsAllocated", "PixelData"):
        if k not in ds:
            raise DicomError(f"no {k} in the dataset: not an image")
    rows, cols = int(ds["Rows"]), int(ds["Columns"])
    frames = int(ds.get("NumberOfFrames", 1))
    spp = int(ds.get("SamplesPerPixel", 1))
    ba = int(ds["BitsAllocated"])
    bs = int(ds.get("BitsStored", ba))
    signed = int(ds.get("PixelRepresentation", 0)) == 1
    if ba not in (8, 16, 32):
        raise NotImplementedError(f"Bits Allocated {ba} (only 8, 16 and 32 are decoded)")
    dt = np.dtype(("<i" if signed else "<u") + str(ba // 8))
    n = rows * cols * frames * spp
    data = ds["PixelData"]
    if isinstance(data, list):  # encapsulated
        if ds["TransferSyntaxUID"] != RLE_LOSSLESS:
            raise NotImplementedError(f"encapsulated pixel data in transfer syntax "
                                      f"{ds['TransferSyntaxUID']}: decoding it needs a codec")
        data = _rle_frames(data[1:], frames, rows, cols, spp, ba // 8)
        spp_planar = True
    else:
        spp_planar = int(ds.get("PlanarConfiguration", 0)) == 1
    if len(data) < n * dt.itemsize:
        raise DicomError(f"PixelData holds {len(data)} bytes, the image needs {n * dt.itemsize}")
    arr = np.frombuffer(data, dtype=dt, count=n).copy()
    if signed and bs < ba:  # sign-extend from Bits Stored
        shift = ba - bs
        arr = ((arr << shift) >> shift).astype(dt)
    if spp > 1:
        if spp_planar:
            arr = arr.reshape(frames, spp, rows, cols).transpose(0, 2, 3, 1)
        else:
            arr = arr.reshape(frames, rows, cols, spp)
    else:
        arr = arr.reshape(frames, rows, cols)
    return np.ascontiguousarray(arr[0] if frames == 1 else arr)


def _unpackbits(seg: bytes, n: int) -> bytes:
    """One RLE segment (PS3.5 G.3.1, PackBits): header byte h < 128 copies the next h + 1
    bytes, 129 .. 255 (-127 .. -1) repeats the next byte 257 - h times, 128 is a no-op;
    the first n bytes of the output (a segment may carry one padding byte)."""
    out = bytearray()
    i, L = 0, len(seg)
    while i < L and len(out) < n:
        h = seg[i]
        i += 1
        if h < 128:
            out += seg[i:i + h + 1]
            i += h + 1
        elif h > 128:
            if i >= L:
                break
            out += bytes((seg[i],)) * (257 - h)
            i += 1
    if len(out) < n:
        raise DicomError(f"RLE segment decodes to {len(out)} bytes, the frame needs {n}")
    return bytes(out[:n])


def _rle_frames(frags: list, frames: int, rows: int, cols: int, spp: int, nbytes: int) -> bytes:
    """RLE Lossless frames (PS3.5 Annex G) -> little-endian native pixel bytes, samples
    planar (sample-major within each frame): segment s * nbytes + k holds byte k (most
    significant first) of sample s of every pixel."""
    if len(frags) < frames:
        raise DicomError(f"{len(frags)} RLE fragments for {frames} frames")
    npix = rows * cols
    out = bytearray()
    for f in range(frames):
        fr = frags[f]
        if len(fr) < 64:
            raise DicomError("RLE frame shorter than its 64-byte header")
        nseg = struct.unpack_from("<I", fr, 0)[0]
        offs = list(struct.unpack_from("<15I", fr, 4))[:nseg]
        if nseg != spp * nbytes:
            raise DicomError(f"RLE frame has {nseg} segments, expected {spp * nbytes}")
        ends = offs[1:] + [len(fr)]
        planes = np.empty((spp, npix, nbytes), dtype=np.uint8)
        for sidx in range(nseg):
            seg = _unpackbits(fr[offs[sidx]:ends[sidx]], npix)
            s_, k = divmod(sidx, nbytes)
            planes[s_, :, nbytes - 1 - k] = np.frombuffer(seg, dtype=np.uint8)
        out += planes.tobytes()
    return bytes(out)
