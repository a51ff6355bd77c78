"""open3d.visualization: only the module path Open3D-ML's pipelines import
(semantic_segmentation.py:13, object_detection.py:13); the GUI and 3D
TensorBoard plugin are out of scope."""
from . import tensorboard_plugin  # noqa: F401
