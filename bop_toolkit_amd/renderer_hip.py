"""RendererHIP — depth renderer plugin backed by the gfx950 rasteriser.

Implements the Renderer interface of bop_toolkit_lib/renderer.py:11-74 for
mode='depth' (the mode eval_calc_errors.py:188-191 uses for VSD/CUS). It
replaces the OpenGL depth pass of renderer_vispy.py:433-538 /
renderer_py.py:422-555: eye-space Z per pixel, sampled at pixel centres,
no back-face culling, nearest surface wins, 0 = background (raster spec:
DESIGN.md §4).

Objects live in the libbopx context's HBM registry, so pose_error.vsd called
with this renderer never moves depth maps over PCIe: both renders are fused
into the VSD kernel.
"""
import numpy as np

from . import inout
from . import runtime
from ._lib import _d, _f, ptr
from .renderer import Renderer


class RendererHIP(Renderer):
  """GPU depth renderer (renderer_type='hip')."""

  def __init__(self, width, height, mode="depth", shading="phong", bg_color=(0.0, 0.0, 0.0, 0.0)):
    super().__init__(width, height)
    if mode != "depth":
      raise NotImplementedError(
          "RendererHIP renders depth only (mode='depth'); RGB shading is outside the "
          "pose-error path")
    self.mode = mode
    self.ctx = runtime.context()
    self.models = {}

  def add_object(self, obj_id, model_path, **kwargs):
    """Load a PLY model (inout.load_ply) and upload it (renderer.py:47-53)."""
    model = inout.load_ply(model_path)
    self.add_object_arrays(obj_id, model["pts"], model.get("faces"))

  def add_object_arrays(self, obj_id, pts, faces):
    """Register an in-memory mesh: pts V x 3, faces F x 3."""
    self.ctx.add_object(obj_id, pts, faces)
    self.models[obj_id] = {"pts": np.asarray(pts), "faces": np.asarray(faces)}

  def remove_object(self, obj_id):
    self.ctx.remove_object(obj_id)
    del self.models[obj_id]

  def render_object(self, obj_id, R, t, fx, fy, cx, cy):
    """{'depth': H x W float32} of obj_id in pose (R, t) (renderer.py:62-74)."""
    R = np.ascontiguousarray(R, np.float64).reshape(9)
    t = np.ascontiguousarray(t, np.float64).reshape(3)
    depth = np.empty((self.height, self.width), np.float32)
    self.ctx.call("bopx_render_depth", int(obj_id), ptr(R, _d), ptr(t, _d), float(fx),
                  float(fy), float(cx), float(cy), self.width, self.height, ptr(depth, _f))
    return {"depth": depth}
