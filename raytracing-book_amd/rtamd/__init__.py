"""rtamd — MI355X-native path-tracing hot path of Bowen951209/raytracing-book.

Layers:
  * rtamd.scene   — host scene builder bindings (Scene.java + RaytraceModel.java mirror)
  * rtamd.render  — rt.h context + RaytraceExecutor mirror
  * rtamd.dist    — one-process-per-GPU stripe partition + RCCL gather
The compute path is the HIP kernel in lib/librtamd.so; nothing here computes pixels.
"""
from ._lib import RTError, amd, amd_ab, scene_lib  # noqa: F401
from .render import (OPTIONS, RaytraceExecutor, RenderContext, comm_unique_id, deinterleave,  # noqa: F401
                     frame_rand_factors,
                     local_rows, padded_local_rows, sah_bvh, stripe_rows_of)
from .scene import SCENE_NAMES, Scene, SceneBuilder, decode_image, save_png, spp_uniforms, tonemap_rgb8  # noqa: F401
