"""Capture golden outputs of the reference PLY reader (bop_toolkit_lib/inout.py
load_ply, inout.py:401-583) on small PLY files written here.

Runs ONLY in the build container (imports /root/reference/bop_toolkit_lib with
the harness stubs of SURVEY.md §8c: imageio/png modules, np.float). Writes the
PLY inputs to tests/golden/ply/ and the reference's parsed arrays to
tests/golden/ply/expected.npz (file name + key), plus the error messages the
reference raises on non-triangular / bad-texcoord faces to expected.json.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_ply.py
"""
import json
import os
import struct
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ply")
REF = os.environ.get("BOP_REFERENCE", "/root/reference")


def _stubs():
  np.float = float
  sys.modules["imageio"] = types.ModuleType("imageio")
  sys.modules["png"] = types.ModuleType("png")
  sys.path.insert(0, REF)


def _header(fmt, nv, vprops, nf, fprops, comment=None):
  h = ["ply", "format %s 1.0" % fmt]
  if comment:
    h.append(comment)
  h.append("element vertex %d" % nv)
  h += ["property %s %s" % (t, n) for n, t in vprops]
  if nf is not None:
    h.append("element face %d" % nf)
    h += fprops
  h.append("end_header")
  return ("\n".join(h) + "\n").encode()


def write_cases(rng):
  os.makedirs(OUT, exist_ok=True)
  nv, nf = 7, 5
  pts = rng.uniform(-50, 50, (nv, 3)).astype(np.float32)
  nrm = rng.uniform(-1, 1, (nv, 3)).astype(np.float32)
  col = rng.integers(0, 256, (nv, 3)).astype(np.uint8)
  uv = rng.uniform(0, 1, (nv, 2)).astype(np.float32)
  faces = rng.integers(0, nv, (nf, 3)).astype(np.int32)
  fuv = rng.uniform(0, 1, (nf, 6)).astype(np.float32)
  cases = {}
  # 1. binary: normals, colours, per-vertex UV, faces + per-face texcoord, texture file
  vp = [("x", "float"), ("y", "float"), ("z", "float"), ("nx", "float"), ("ny", "float"),
        ("nz", "float"), ("red", "uchar"), ("green", "uchar"), ("blue", "uchar"),
        ("texture_u", "float"), ("texture_v", "float")]
  fp = ["property list uchar int vertex_indices", "property list uchar float texcoord"]
  b = bytearray(_header("binary_little_endian", nv, vp, nf, fp, "comment TextureFile tex.png"))
  for i in range(nv):
    b += struct.pack("<6f3B2f", *pts[i], *nrm[i], *col[i], *uv[i])
  for i in range(nf):
    b += struct.pack("<B3iB6f", 3, *faces[i], 6, *fuv[i])
  cases["full_binary.ply"] = bytes(b)
  # 2. binary, double vertices, plain faces
  b = bytearray(_header("binary_little_endian", nv, [("x", "double"), ("y", "double"),
                                                     ("z", "double")], nf,
                        ["property list uchar int vertex_indices"]))
  for i in range(nv):
    b += struct.pack("<3d", *pts[i].astype(np.float64) / 3.0)
  for i in range(nf):
    b += struct.pack("<B3i", 3, *faces[i])
  cases["double_binary.ply"] = bytes(b)
  # 3. ascii with normals and faces
  t = _header("ascii", nv, vp[:6], nf, ["property list uchar int vertex_indices"]).decode()
  t += "".join("%r %r %r %r %r %r\n" % tuple(float(x) for x in np.r_[pts[i], nrm[i]])
               for i in range(nv))
  t += "".join("3 %d %d %d\n" % tuple(faces[i]) for i in range(nf))
  cases["normals_ascii.ply"] = t.encode()
  # 4. points only (no face element)
  b = bytearray(_header("binary_little_endian", nv, vp[:3], None, None))
  for i in range(nv):
    b += struct.pack("<3f", *pts[i])
  cases["points_only.ply"] = bytes(b)
  # 5. error cases: a quad face, a texcoord list of 4 values
  b = bytearray(_header("binary_little_endian", 4, vp[:3], 1,
                        ["property list uchar int vertex_indices"]))
  for i in range(4):
    b += struct.pack("<3f", *pts[i])
  b += struct.pack("<B4i", 4, 0, 1, 2, 3)
  cases["err_quad.ply"] = bytes(b)
  b = bytearray(_header("binary_little_endian", 3, vp[:3], 1, fp))
  for i in range(3):
    b += struct.pack("<3f", *pts[i])
  b += struct.pack("<B3iB4f", 3, 0, 1, 2, 4, 0.1, 0.2, 0.3, 0.4)
  cases["err_texcoord.ply"] = bytes(b)
  for name, data in cases.items():
    with open(os.path.join(OUT, name), "wb") as f:
      f.write(data)
  return sorted(cases)


def main():
  names = write_cases(np.random.default_rng(11))
  _stubs()
  from bop_toolkit_lib import inout as ref_inout
  arrays, meta = {}, {}
  for name in names:
    try:
      m = ref_inout.load_ply(os.path.join(OUT, name))
    except ValueError as e:
      meta[name] = {"error": str(e)}
      continue
    meta[name] = {"keys": sorted(m), "texture_file": m.get("texture_file")}
    for k, v in m.items():
      if isinstance(v, np.ndarray):
        arrays["%s|%s" % (name, k)] = v
  np.savez(os.path.join(OUT, "expected.npz"), **arrays)
  with open(os.path.join(OUT, "expected.json"), "w") as f:
    json.dump(meta, f, indent=1, sort_keys=True)
  print(json.dumps(meta, indent=1))


if __name__ == "__main__":
  main()
