"""Renderer plugin interface (mirror of bop_toolkit_lib/renderer.py:11-104).

The factory adds renderer_type='hip' (RendererHIP, the gfx950 rasteriser).
The reference's OpenGL back-ends ('vispy', 'python') and the external C++
'cpp' renderer are not part of this package. For an import-only drop-in
(scripts/eval_calc_errors.py:57 defaults renderer_type='vispy' and calls
create_renderer(W, H, p['renderer_type'], mode='depth') at :188-189), the
environment variable BOPX_RENDERER_ALIAS names reference back-ends (comma
separated, e.g. "vispy" or "vispy,cpp,python") that the factory maps to
RendererHIP. It is opt-in: without it those names raise as before, so nobody
gets a different rasteriser than the one they asked for by accident.
"""
import os


class Renderer(object):
  """Abstract renderer (renderer.py:11-74)."""

  def __init__(self, width, height):
    self.width = width
    self.height = height
    self.light_cam_pos = (0, 0, 0)
    self.light_color = (1.0, 1.0, 1.0)
    self.light_ambient_weight = 0.5
    self.light_diffuse_weight = 1.0
    self.light_specular_weight = 0.0
    self.light_specular_shininess = 0.0

  def set_light_cam_pos(self, light_cam_pos):
    self.light_cam_pos = light_cam_pos

  def set_light_ambient_weight(self, light_ambient_weight):
    self.light_ambient_weight = light_ambient_weight

  def add_object(self, obj_id, model_path, **kwargs):
    raise NotImplementedError

  def remove_object(self, obj_id):
    raise NotImplementedError

  def render_object(self, obj_id, R, t, fx, fy, cx, cy):
    raise NotImplementedError


def create_renderer(width, height, renderer_type="hip", mode="depth", shading="phong",
                    bg_color=(0.0, 0.0, 0.0, 0.0)):
  """Renderer factory (renderer.py:77-104) with the 'hip' back-end."""
  alias = {a.strip() for a in os.environ.get("BOPX_RENDERER_ALIAS", "").split(",") if a.strip()}
  if renderer_type == "hip" or renderer_type in alias:
    from .renderer_hip import RendererHIP
    return RendererHIP(width, height, mode, shading, bg_color)
  if renderer_type in ("vispy", "python", "cpp"):
    raise NotImplementedError(
        "renderer_type=%r is an OpenGL/C++ back-end of bop_toolkit_lib; use "
        "renderer_type='hip'" % (renderer_type,))
  raise ValueError("Unknown renderer type.")
