"""Host I/O needed around the pose-error path (subset of bop_toolkit_lib/inout.py).

load_ply reads the vertices and triangles of a BOP model (inout.py:401-583
parses them with a per-vertex Python loop; here the binary body is decoded
with one structured-dtype read). Other per-vertex attributes are skipped.
"""
import json

import numpy as np

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1",
    "short": "i2", "int16": "i2", "ushort": "u2", "uint16": "u2",
    "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


def _read_header(f):
  elements, fmt = [], None
  line = f.readline().strip()
  if line != b"ply":
    raise ValueError("not a PLY file")
  while True:
    line = f.readline()
    if not line:
      raise ValueError("truncated PLY header")
    tok = line.decode("ascii", "replace").split()
    if not tok:
      continue
    if tok[0] == "format":
      fmt = tok[1]
    elif tok[0] == "element":
      elements.append({"name": tok[1], "count": int(tok[2]), "props": []})
    elif tok[0] == "property":
      if tok[1] == "list":
        elements[-1]["props"].append((tok[4], "list", _PLY_TYPES[tok[2]], _PLY_TYPES[tok[3]]))
      else:
        elements[-1]["props"].append((tok[2], "scalar", _PLY_TYPES[tok[1]], None))
    elif tok[0] == "end_header":
      return fmt, elements


def load_ply(path):
  """Returns {'pts': V x 3 float64, 'faces': F x 3 int64}."""
  with open(path, "rb") as f:
    fmt, elements = _read_header(f)
    body = f.read()
  if fmt == "ascii":
    return _load_ascii(body.decode("ascii").split("\n"), elements)
  if fmt != "binary_little_endian":
    raise ValueError("unsupported PLY format %r" % fmt)
  off, pts, faces = 0, None, None
  for el in elements:
    n = el["count"]
    if all(p[1] == "scalar" for p in el["props"]):
      dt = np.dtype([(p[0], "<" + p[2]) for p in el["props"]])
      arr = np.frombuffer(body, dt, count=n, offset=off)
      off += n * dt.itemsize
      if el["name"] == "vertex":
        pts = np.stack([arr["x"], arr["y"], arr["z"]], 1).astype(np.float64)
    elif el["name"] == "face" and len(el["props"]) == 1:
      _, _, ct, it = el["props"][0]
      cdt, idt = np.dtype("<" + ct), np.dtype("<" + it)
      first = int(np.frombuffer(body, cdt, count=1, offset=off)[0]) if n else 3
      dt = np.dtype([("n", cdt), ("i", idt, (first,))])
      arr = np.frombuffer(body, dt, count=n, offset=off)
      if n and not np.all(arr["n"] == first):
        raise ValueError("mixed polygon sizes are not supported")
      if first != 3 and n:
        raise ValueError("only triangle meshes are supported")
      faces = arr["i"].astype(np.int64)
      off += n * dt.itemsize
    else:
      raise ValueError("unsupported PLY element layout %r" % el["name"])
  return {"pts": pts, "faces": faces if faces is not None else np.zeros((0, 3), np.int64)}


def _load_ascii(lines, elements):
  pos, pts, faces = 0, None, None
  for el in elements:
    rows = [l.split() for l in lines[pos:pos + el["count"]]]
    pos += el["count"]
    if el["name"] == "vertex":
      names = [p[0] for p in el["props"]]
      a = np.array(rows, np.float64)
      pts = a[:, [names.index("x"), names.index("y"), names.index("z")]]
    elif el["name"] == "face":
      faces = np.array([[int(v) for v in r[1:4]] for r in rows], np.int64).reshape(-1, 3)
  return {"pts": pts, "faces": faces if faces is not None else np.zeros((0, 3), np.int64)}


def save_ply(path, pts, faces):
  """Minimal binary PLY writer (vertices as float32, triangles as int32)."""
  pts = np.asarray(pts, np.float32)
  faces = np.asarray(faces, np.int32)
  head = ("ply\nformat binary_little_endian 1.0\nelement vertex %d\n"
          "property float x\nproperty float y\nproperty float z\n"
          "element face %d\nproperty list uchar int vertex_indices\nend_header\n"
          % (len(pts), len(faces)))
  fdt = np.dtype([("n", "u1"), ("i", "<i4", (3,))])
  farr = np.empty(len(faces), fdt)
  farr["n"] = 3
  farr["i"] = faces
  with open(path, "wb") as f:
    f.write(head.encode("ascii"))
    f.write(pts.astype("<f4").tobytes())
    f.write(farr.tobytes())


def _make_dumps():
  """json.dumps(o, sort_keys=True) without the per-call encoder set-up: one C
  encoder (the one json.dumps itself builds for every call) reused for every
  element. Same bytes: same separators, float repr, ASCII escaping, NaN/inf."""
  from json import encoder as je
  if getattr(je, "c_make_encoder", None) is None:
    return json.JSONEncoder(sort_keys=True).encode

  def default(o):
    raise TypeError("Object of type {} is not JSON serializable".format(type(o).__name__))

  enc = je.c_make_encoder(None, default, je.encode_basestring_ascii, None, ": ", ", ", True,
                          False, True)

  def dumps(o):
    if isinstance(o, str):
      return je.encode_basestring_ascii(o)
    return "".join(enc(o, 0))
  return dumps


_dumps = _make_dumps()


def save_json(path, content):
  """JSON with one top-level element per line and sorted keys
  (inout.py:85-113), the format of the errors_*.json hand-off files."""
  with open(path, "w") as f:
    if isinstance(content, dict):
      items = sorted(content.items(), key=lambda x: x[0])
      body = ",\n".join('  "{}": {}'.format(k, _dumps(v)) for k, v in items)
      f.write("{\n" + body + ("\n}" if items else "}"))
    elif isinstance(content, list):
      body = ",\n".join("  " + _dumps(e) for e in content)
      f.write("[\n" + body + ("\n]" if content else "]"))
    else:
      json.dump(content, f, sort_keys=True)


def load_json(path, keys_to_int=False):
  """JSON file; with keys_to_int, object keys that are (signed) integers
  become ints (inout.py:66-82)."""
  def hook(d):
    return {int(k) if k.lstrip("-").isdigit() else k: v for k, v in d.items()}
  with open(path, "r") as f:
    return json.load(f, object_hook=hook) if keys_to_int else json.load(f)


def load_depth(path):
  """16-bit depth image (PNG, or TIFF for ITODD) as float32 (inout.py:39-46;
  the reference reads it with imageio, here with Pillow)."""
  from PIL import Image
  with Image.open(path) as im:
    return np.asarray(im).astype(np.float32)


def load_cam_params(path):
  """im_size (w, h), K and optional depth_scale of a camera.json (inout.py:116-137)."""
  c = load_json(path)
  cam = {"im_size": (c["width"], c["height"]),
         "K": np.array([[c["fx"], 0.0, c["cx"]], [0.0, c["fy"], c["cy"]], [0.0, 0.0, 1.0]])}
  if "depth_scale" in c:
    cam["depth_scale"] = float(c["depth_scale"])
  return cam


def _as(d, key, shape):
  if key in d:
    d[key] = np.array(d[key], np.float64).reshape(shape)


def load_scene_camera(path):
  """scene_camera.json: per image cam_K (3x3), cam_R_w2c, cam_t_w2c as float64
  arrays, other fields as stored (inout.py:140-160)."""
  scene_camera = load_json(path, keys_to_int=True)
  for cam in scene_camera.values():
    _as(cam, "cam_K", (3, 3))
    _as(cam, "cam_R_w2c", (3, 3))
    _as(cam, "cam_t_w2c", (3, 1))
  return scene_camera


def load_scene_gt(path):
  """scene_gt.json: per image a list of GT instances with cam_R_m2c (3x3) and
  cam_t_m2c (3x1) float64 (inout.py:182-198)."""
  scene_gt = load_json(path, keys_to_int=True)
  for im_gt in scene_gt.values():
    for gt in im_gt:
      _as(gt, "cam_R_m2c", (3, 3))
      _as(gt, "cam_t_m2c", (3, 1))
  return scene_gt


def load_bop_results(path, version="bop19"):
  """BOP19 CSV results: scene_id,im_id,obj_id,score,R,t,time; a first line
  containing the header is skipped (inout.py:221-261)."""
  if version != "bop19":
    raise ValueError("Unknown version of BOP results.")
  header = "scene_id,im_id,obj_id,score,R,t,time"
  results = []
  with open(path, "r") as f:
    for line_no, line in enumerate(f, 1):
      if line_no == 1 and header in line:
        continue
      e = line.split(",")
      if len(e) != 7:
        raise ValueError("A line does not have 7 comma-sep. elements: {}".format(line))
      results.append({
          "scene_id": int(e[0]), "im_id": int(e[1]), "obj_id": int(e[2]),
          "score": float(e[3]),
          "R": np.array([float(x) for x in e[4].split()], np.float64).reshape((3, 3)),
          "t": np.array([float(x) for x in e[5].split()], np.float64).reshape((3, 1)),
          "time": float(e[6])})
  return results


def load_depths(paths, workers=None):
  """load_depth of many files, decoded in a thread pool (Pillow's PNG/TIFF
  decoders release the GIL), in input order."""
  from concurrent.futures import ThreadPoolExecutor
  paths = list(paths)
  if len(paths) <= 1:
    return [load_depth(p) for p in paths]
  import os
  n = workers or min(16, os.cpu_count() or 1, len(paths))
  with ThreadPoolExecutor(n) as pool:
    return list(pool.map(load_depth, paths))
