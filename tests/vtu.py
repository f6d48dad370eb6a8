"""Minimal reader for the appended-base64 .vtu files the drivers write
(VTK XML UnstructuredGrid, UInt32 headers, header and payload base64-encoded
separately).  Test helper only."""
import base64
import re

import numpy as np

_DT = {"Float64": np.float64, "Float32": np.float32, "Int64": np.int64, "UInt8": np.uint8}


def read_vtu(path):
    text = open(path).read()
    start = text.index("<AppendedData")
    data = text[text.index("_", start) + 1:]
    arrays = {}
    for m in re.finditer(r'<DataArray type="(\w+)" Name="(\w+)"[^>]*offset="(\d+)"', text[:start]):
        typ, name, off = m.group(1), m.group(2), int(m.group(3))
        nbytes = int(np.frombuffer(base64.b64decode(data[off:off + 8]), dtype=np.uint32)[0])
        nchar = (nbytes + 2) // 3 * 4
        raw = base64.b64decode(data[off + 8:off + 8 + nchar]) if nbytes else b""
        arrays[name] = np.frombuffer(raw, dtype=_DT[typ])
    npts = int(re.search(r'NumberOfPoints="(\d+)"', text).group(1))
    return npts, arrays
