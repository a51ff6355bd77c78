"""Drop-in for ``open3d.ml.torch.layers`` on the hot path."""
import torch

from . import ops


class FixedRadiusSearch(torch.nn.Module):
    """Open3D ``layers.FixedRadiusSearch`` (kpconv.py:2021-2023): builds the
    spatial hash table (unless one is given) and runs fixed_radius_search."""

    def __init__(self, metric="L2", ignore_query_point=False, return_distances=False,
                 max_hash_table_size=32 * 2**20, index_dtype=torch.int32, **kwargs):
        super().__init__()
        self.metric = metric
        self.ignore_query_point = ignore_query_point
        self.return_distances = return_distances
        self.max_hash_table_size = max_hash_table_size
        self.index_dtype = index_dtype

    def forward(self, points, queries, radius, points_row_splits=None, queries_row_splits=None,
                hash_table_size_factor=1 / 64, hash_table=None):
        if points_row_splits is None:
            points_row_splits = torch.LongTensor([0, points.shape[0]])
        if queries_row_splits is None:
            queries_row_splits = torch.LongTensor([0, queries.shape[0]])
        if hash_table is None:
            table = ops.build_spatial_hash_table(points, radius, points_row_splits,
                                                 hash_table_size_factor,
                                                 max_hash_table_size=self.max_hash_table_size)
        else:
            table = hash_table
        return ops.fixed_radius_search(points, queries, radius, points_row_splits, queries_row_splits,
                                       hash_table_splits=table.hash_table_splits,
                                       hash_table_index=table.hash_table_index,
                                       hash_table_cell_splits=table.hash_table_cell_splits,
                                       index_dtype=self.index_dtype, metric=self.metric,
                                       ignore_query_point=self.ignore_query_point,
                                       return_distances=self.return_distances)


class KNNSearch(torch.nn.Module):
    """Open3D ``layers.KNNSearch`` (point_transformer.py:724-729)."""

    def __init__(self, metric="L2", ignore_query_point=False, return_distances=False,
                 index_dtype=torch.int32, **kwargs):
        super().__init__()
        self.metric = metric
        self.ignore_query_point = ignore_query_point
        self.return_distances = return_distances
        self.index_dtype = index_dtype

    def forward(self, points, queries, k, points_row_splits=None, queries_row_splits=None):
        if points_row_splits is None:
            points_row_splits = torch.LongTensor([0, points.shape[0]])
        if queries_row_splits is None:
            queries_row_splits = torch.LongTensor([0, queries.shape[0]])
        return ops.knn_search(points, queries, k, points_row_splits, queries_row_splits,
                              index_dtype=self.index_dtype, metric=self.metric,
                              ignore_query_point=self.ignore_query_point,
                              return_distances=self.return_distances)
