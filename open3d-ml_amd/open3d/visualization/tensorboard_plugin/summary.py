"""open3d.visualization.tensorboard_plugin.summary: imported by the reference
pipelines (semantic_segmentation.py:13, object_detection.py:17) for 3D
TensorBoard summaries, which this build does not provide (SURVEY.md §2.2,
OUT OF SCOPE).  Importing works; writing a 3D summary raises."""


def add_3d(*args, **kwargs):
    raise NotImplementedError("Open3D's 3D TensorBoard summaries are not part of o3dml_amd (SURVEY.md §2.2)")
