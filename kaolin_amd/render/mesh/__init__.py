"""Mirror of kaolin/render/mesh/__init__.py (hot-path functions)."""
from .rasterization import rasterize, rasterize_from_rast  # noqa: F401
from .dibr import (dibr_soft_mask, dibr_rasterization, dibr_rasterization_from_vertices,  # noqa: F401
                   dibr_rasterization_with_mask_iou)
from .utils import prepare_vertices, texture_mapping  # noqa: F401
from .deftet import deftet_sparse_render  # noqa: F401
