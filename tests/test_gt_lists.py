"""Native scene_gt / scene_gt_info reader (bopx_gt_lists_open, include/bopx_io.h)
against the Python JSON path (inout.load_scene_gt / load_json): the same
images, records and float64 values on the files it takes, and a decline (None)
on every file outside its strict form, so the caller's json parse meets what
the reference meets."""
import json
import os

import numpy as np
import pytest

from bop_toolkit_amd import inout

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _check_gt(path):
  g = inout.load_scene_gt_lists(path)
  d = inout.load_scene_gt(path)
  assert g is not None
  assert g.im_ids.tolist() == list(d)
  for im, lst in d.items():
    a, b = g.rows(im)
    assert b - a == len(lst)
    for k, gt in enumerate(lst):
      assert np.array_equal(gt["cam_R_m2c"].reshape(9).view(np.uint64),
                            g.fields["cam_R_m2c"][a + k].view(np.uint64))
      assert np.array_equal(gt["cam_t_m2c"].reshape(3).view(np.uint64),
                            g.fields["cam_t_m2c"][a + k].view(np.uint64))
      assert gt["obj_id"] == g.obj[a + k]
  return g


def test_golden_scene_files():
  found = 0
  for root, _, files in os.walk(GOLDEN):
    for f in files:
      p = os.path.join(root, f)
      if f.endswith("scene_gt.json"):
        _check_gt(p)
        found += 1
      elif f.endswith("scene_gt_info.json"):
        g = inout.load_scene_gt_info_lists(p)
        d = inout.load_json(p, keys_to_int=True)
        assert g is not None and g.im_ids.tolist() == list(d)
        for im, lst in d.items():
          a, b = g.rows(im)
          assert [x["visib_fract"] for x in lst] == g.fields["visib_fract"][a:b, 0].tolist()
        found += 1
  if not found:
    pytest.skip("no scene files in tests/golden")


def _numbers(rng, n):
  """Decimal spellings json and float() must agree on: ints, exponents,
  17-digit mantissas, subnormals, huge values, negative zero."""
  out = []
  for _ in range(n):
    k = int(rng.integers(0, 8))
    if k == 0:
      out.append(str(int(rng.integers(-10 ** 6, 10 ** 6))))
    elif k == 1:
      out.append(repr(float(rng.normal() * 10 ** int(rng.integers(-30, 30)))))
    elif k == 2:
      out.append("%.17e" % float(rng.normal()))
    elif k == 3:
      out.append("%dE%+d" % (int(rng.integers(1, 99)), int(rng.integers(-330, 330))))
    elif k == 4:
      out.append("-0.0")
    elif k == 5:
      out.append("4.9e-324")
    elif k == 6:
      out.append("1e400")
    else:
      out.append("0.%s" % "".join(str(int(x)) for x in rng.integers(0, 10, 25)))
  return out


def test_random_files_bitwise(tmp_path):
  rng = np.random.default_rng(5)
  for case in range(20):
    parts = []
    for im in rng.permutation(int(rng.integers(0, 40))).tolist():
      recs = []
      for _ in range(int(rng.integers(0, 7))):
        R, t = _numbers(rng, 9), _numbers(rng, 3)
        fields = ['"cam_R_m2c": [%s]' % ", ".join(R), '"cam_t_m2c": [%s]' % ",".join(t),
                  '"obj_id": %d' % int(rng.integers(1, 30))]
        if rng.random() < 0.3:
          fields.append('"extra": {"a": [1, "x\\"y", null, true, false, {}], "b": []}')
        rng.shuffle(fields)
        recs.append("{%s}" % (",\n " if rng.random() < 0.5 else ", ").join(fields))
      parts.append('"%d": [%s]' % (im, ", ".join(recs)))
    p = tmp_path / ("g%d.json" % case)
    p.write_text("{\n" + ",\n".join(parts) + "\n}\n")
    _check_gt(str(p))


@pytest.mark.parametrize("text", [
    '{"1": [{"cam_R_m2c": [1,2,3,4,5,6,7,8,9], "cam_t_m2c": [1,2,3]}]}',  # no obj_id
    '{"1": [{"cam_R_m2c": [1,2,3,4,5,6,7,8], "cam_t_m2c": [1,2,3], "obj_id": 1}]}',
    '{"1": [{"cam_R_m2c": [1,2,3,4,5,6,7,8,NaN], "cam_t_m2c": [1,2,3], "obj_id": 1}]}',
    '{"1": [{"cam_R_m2c": [1,2,3,4,5,6,7,8,9], "cam_t_m2c": [1,2,3], "obj_id": 1.5}]}',
    '{"1": [{"cam_R_m2c": [1,2,3,4,5,6,7,8,9], "cam_t_m2c": [1,2,3], "obj_id": true}]}',
    '{"1": [{"cam_R_m2c": [1,2,3,4,5,6,7,8,9], "cam_t_m2c": [1,2,3], "obj_id": 1, "obj_id": 2}]}',
    '{"1": [], "01": []}',  # two keys for image 1
    '{"a": []}',
    '{"1": {}}',
    '{"1": [{"cam_R_m2c": [1,2,3,4,5,6,7,8,9], "cam_t_m2c": [1,2,3], "obj_id": 01}]}',
    '{"1": [{"cam_R_m2c": [[1,2,3],[4,5,6],[7,8,9]], "cam_t_m2c": [1,2,3], "obj_id": 1}]}',
    '{"1": []',
    '{"1": []} x',
    '﻿{"1": []}',
    '{"\\u0031": []}',
])
def test_declined(tmp_path, text):
  p = tmp_path / "scene_gt.json"
  p.write_text(text, encoding="utf-8")
  assert inout.load_scene_gt_lists(str(p)) is None


def test_empty_and_missing(tmp_path):
  p = tmp_path / "scene_gt.json"
  p.write_text(" { } ")
  g = inout.load_scene_gt_lists(str(p))
  assert g is not None and len(g.im_ids) == 0 and g.off.tolist() == [0]
  with pytest.raises(KeyError):
    g.rows(3)
  assert inout.load_scene_gt_lists(str(tmp_path / "missing.json")) is None


def test_arrays_path_matches_dict_path(tmp_path):
  """scene_arrays_direct on the GTLists gives the dict path's arrays."""
  from bop_toolkit_amd import eval_calc_errors as ece
  rng = np.random.default_rng(11)
  scene_gt, targets, ests = {}, {}, {}
  for im in range(30):
    objs = rng.choice(np.arange(1, 8), int(rng.integers(1, 5)), replace=True).tolist()
    scene_gt[str(im)] = [{"cam_R_m2c": rng.normal(size=9).tolist(),
                          "cam_t_m2c": (rng.normal(size=3) * 100).tolist(), "obj_id": o}
                         for o in objs]
    targets[im] = {o: {"inst_count": objs.count(o)} for o in set(objs)}
    ests[im] = {o: [{"score": float(rng.random()), "R": rng.normal(size=(3, 3)),
                     "t": rng.normal(size=(3, 1))} for _ in range(int(rng.integers(0, 4)))]
                for o in set(objs)}
  p = tmp_path / "scene_gt.json"
  p.write_text(json.dumps(scene_gt))
  prm = {"n_top": -1, "skip_missing": True}
  a0, n0 = ece.scene_arrays_direct(prm, 1, targets, {1: ests}, inout.load_scene_gt(str(p)))
  a1, n1 = ece.scene_arrays_direct(prm, 1, targets, {1: ests}, inout.load_scene_gt_lists(str(p)))
  assert n0 == n1
  for k in a0:
    assert np.array_equal(a0[k], a1[k]), k


_GOOD_REC = '"cam_R_m2c": [1,2,3,4,5,6,7,8,9], "cam_t_m2c": [1,2,3], "obj_id": 1'


@pytest.mark.parametrize("raw", [
    ('{"1": [{%s, "x": "a\\qb"}]}' % _GOOD_REC).encode(),  # unknown escape
    ('{"1": [{%s, "x": "a\\u12"}]}' % _GOOD_REC).encode(),  # short \u escape
    ('{"1": [{%s, "x": "a\\u12G4"}]}' % _GOOD_REC).encode(),  # not hex
    ('{"1": [{%s, "x": "a\\' % _GOOD_REC).encode(),  # escape at the end of the file
    ('{"1": [{%s, "x": "' % _GOOD_REC).encode() + b'\xff"}]}',  # not UTF-8
    ('{"1": [{%s, "x": "' % _GOOD_REC).encode() + b'\xc3"}]}',  # truncated sequence
    ('{"1": [{%s, "x": "' % _GOOD_REC).encode() + b'\xed\xa0\x80"}]}',  # a surrogate
    ('{"1": [{%s, "x": "' % _GOOD_REC).encode() + b'\xc0\xaf"}]}',  # overlong form
])
def test_declined_bad_strings(tmp_path, raw):
  """text Python's json (as the reference opens it, inout.py:66-82)
  refuses is declined, so the Python path raises the reference's error."""
  import json
  p = tmp_path / "scene_gt.json"
  p.write_bytes(raw)
  assert inout.load_scene_gt_lists(str(p)) is None
  with pytest.raises(ValueError):  # JSONDecodeError and UnicodeDecodeError are ValueErrors
    with open(str(p), "r", encoding="utf-8") as f:
      json.load(f)


@pytest.mark.parametrize("member", ['"a\\"b\\\\c\\/d\\b\\f\\n\\r\\t"', '"\\u00e9\\uD83D\\ude00"',
                                    '"' + "é中\U0001f600" + '"'])
def test_taken_escapes_and_utf8(tmp_path, member):
  """Every JSON escape and well-formed multi-byte UTF-8 in a skipped member is
  taken, with the same values as the json path."""
  p = tmp_path / "scene_gt.json"
  p.write_text('{"1": [{%s, "x": %s}], "2": []}' % (_GOOD_REC, member), encoding="utf-8")
  g = inout.load_scene_gt_lists(str(p))
  assert g is not None and g.im_ids.tolist() == [1, 2]
  _check_gt(str(p))
