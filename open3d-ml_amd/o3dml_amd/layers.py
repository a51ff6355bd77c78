"""Drop-in for ``open3d.ml.torch.layers`` on the hot path."""
import numpy as np
import torch

from . import ops
from . import sparse_conv as sc


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
        if hash_table is None:  # table build + search in one library call
            return ops._fixed_radius_search_layer(points, queries, radius, points_row_splits, queries_row_splits,
                                                  hash_table_size_factor, self.max_hash_table_size,
                                                  self.index_dtype, self.metric, self.ignore_query_point,
                                                  self.return_distances)
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


class RadiusSearch(torch.nn.Module):
    """Open3D ``layers.RadiusSearch`` (per-query radii; Open3D ml API,
    SURVEY §2.2): ops.radius_search with the layer's options."""

    def __init__(self, metric="L2", ignore_query_point=False, return_distances=False,
                 normalize_distances=False, index_dtype=torch.int32, **kwargs):
        super().__init__()
        self.metric = metric
        self.ignore_query_point = ignore_query_point
        self.return_distances = return_distances
        self.normalize_distances = normalize_distances
        self.index_dtype = index_dtype

    def forward(self, points, queries, radii, points_row_splits=None, queries_row_splits=None):
        if points_row_splits is None:
            points_row_splits = torch.LongTensor([0, points.shape[0]])
        if queries_row_splits is None:
            queries_row_splits = torch.LongTensor([0, queries.shape[0]])
        return ops.radius_search(points, queries, radii, points_row_splits, queries_row_splits,
                                 index_dtype=self.index_dtype, metric=self.metric,
                                 ignore_query_point=self.ignore_query_point,
                                 return_distances=self.return_distances,
                                 normalize_distances=self.normalize_distances)


def _voxel_size_scalar(voxel_size, like):
    if isinstance(voxel_size, torch.Tensor):
        if voxel_size.dim() != 0 and voxel_size.numel() != 1:
            raise Exception("voxel_size must be a scalar")
        return float(voxel_size.reshape(-1)[0])
    return float(voxel_size)


class SparseConv(torch.nn.Module):
    """Open3D ``layers.SparseConv`` (sparseconvnet.py:344-441).

    Neighbours: FixedRadiusSearch(metric='Linf') of the input positions around
    queries out_positions - offset*voxel_size with radius kernel_size*vs/2;
    kernel index of each pair from the relative position; then the MFMA
    gather-GEMM (ops.sparse_conv) with bias/activation.  Parameters:
    ``kernel`` [*kernel_size, Cin, Cout], ``bias`` [Cout], ``offset`` [3]
    (state_dict layout of the reference, load_unet_wts :660-677)."""

    def __init__(self, in_channels, filters, kernel_size, activation=None, use_bias=True,
                 kernel_initializer=torch.nn.init.xavier_uniform_, bias_initializer=torch.nn.init.zeros_,
                 normalize=False, offset=None, max_temp_mem_MB=64, **kwargs):
        super().__init__()
        self.in_channels = in_channels
        self.filters = filters
        self.kernel_size = list(kernel_size)
        if len(set(self.kernel_size)) != 1 or len(self.kernel_size) != 3:
            raise ValueError("SparseConv: only cubic 3-D kernels are supported")
        self.activation = activation
        self.use_bias = use_bias
        self.normalize = normalize
        self.max_temp_mem_MB = max_temp_mem_MB
        if offset is None:
            offset = torch.zeros((3,), dtype=torch.float32)
        self.offset = torch.nn.Parameter(torch.as_tensor(offset, dtype=torch.float32).reshape(3),
                                         requires_grad=False)
        self.kernel = torch.nn.Parameter(torch.empty(*self.kernel_size, in_channels, filters))
        kernel_initializer(self.kernel)
        if use_bias:
            self.bias = torch.nn.Parameter(torch.empty(filters))
            bias_initializer(self.bias)
        else:
            self.bias = None
        self.nns = FixedRadiusSearch(metric="Linf", ignore_query_point=False, return_distances=False)
        self.lattice_rulebook = True  # False forces the fixed-radius-search rulebook

    def _rulebook(self, inp_positions, out_positions, voxel_size, hash_table, mirror, sign):
        sc.note_search_rulebook()
        vs = _voxel_size_scalar(voxel_size, inp_positions)
        queries = (out_positions - sign * self.offset.to(out_positions.device) * vs).contiguous()
        radius = 0.5 * vs * self.kernel_size[0]
        nb = self.nns(inp_positions, queries, radius, hash_table=hash_table)
        kidx = sc.kernel_index(inp_positions, queries, nb.neighbors_index, nb.neighbors_row_splits,
                               self.kernel_size, vs, mirror=mirror)
        self._avg_neighbors = nb.neighbors_index.shape[0] / max(1, out_positions.shape[0])
        return nb, kidx

    def _offset_shift(self, vs, sign):
        """(offset as host floats, query shift or None): queries are
        out_positions - (sign * vs) * offset — the f32 product here, the f32
        subtraction inside the map kernels (the torch expression's bits)."""
        if getattr(self, "_off_ver", None) != (self.offset._version, self.offset.device):
            self._off_host = tuple(float(v) for v in self.offset.detach().cpu())  # one read per load
            self._off_ver = (self.offset._version, self.offset.device)
        off = self._off_host
        return off, (None if not any(off) else tuple(float(np.float32(sign * vs) * np.float32(o)) for o in off))

    def prefetch_map(self, inp_positions, out_positions, voxel_size):
        """Builds this layer's eval-mode lattice map for (inp -> out) on the
        current stream ahead of the layer (sparse_conv.prefetch_lattice_map)."""
        if not self.lattice_rulebook or self.normalize:
            return False
        mirror, sign = (True, -1.0) if isinstance(self, SparseConvTranspose) else (False, 1.0)
        vs = _voxel_size_scalar(voxel_size, inp_positions)
        off, shift = self._offset_shift(vs, sign)
        return sc.prefetch_lattice_map(self.kernel_size[0], inp_positions, out_positions, vs, mirror, sign, off,
                                       shift)

    def _lattice(self, inp_features, inp_positions, out_positions, voxel_size, hash_table, mirror, sign, **kw):
        """Lattice rulebook (same dense map as the Linf search, see
        sparse_conv.conv_lattice) unless a prebuilt search hash table is given."""
        if hash_table is not None or not self.lattice_rulebook:
            return None
        vs = _voxel_size_scalar(voxel_size, inp_positions)
        off, shift = self._offset_shift(vs, sign)
        return sc.conv_lattice(self.kernel, kw.pop("bias", self.bias), inp_features, inp_positions, out_positions, vs,
                               mirror=mirror, cache_key=(inp_positions, out_positions, sign) + off, query_shift=shift,
                               **kw)

    def forward_fused(self, inp_features, inp_positions, out_positions, voxel_size, pre=None, residual=None):
        """Inference form used by SparseConvUnet in eval mode:
        forward(relu(x * pre[0] + pre[1])) + residual with the activation
        applied while the rows are gathered and the residual added in the
        GEMM epilogue (lattice rulebook); unfused otherwise."""
        mirror, sign = (True, -1.0) if isinstance(self, SparseConvTranspose) else (False, 1.0)
        bias = None if mirror else self.bias
        out = None
        if not self.normalize and not (self.activation and residual is not None):
            out = self._lattice(inp_features, inp_positions, out_positions, voxel_size, None, mirror, sign,
                                bias=bias, pre=pre, residual=residual)
        if out is None:
            x = inp_features if pre is None else torch.relu(inp_features * pre[0] + pre[1])
            out = self.forward(x, inp_positions, out_positions, voxel_size)
            return out if residual is None else out + residual
        if mirror and self.bias is not None:
            out = out + self.bias
        return self.activation(out) if self.activation else out

    def forward(self, inp_features, inp_positions, out_positions, voxel_size, inp_importance=None,
                fixed_radius_search_hash_table=None):
        out = self._lattice(inp_features, inp_positions, out_positions, voxel_size, fixed_radius_search_hash_table,
                            False, 1.0, inp_importance=inp_importance, normalize=self.normalize)
        if out is not None:
            return self.activation(out) if self.activation else out
        nb, kidx = self._rulebook(inp_positions, out_positions, voxel_size, fixed_radius_search_hash_table,
                                  False, 1.0)
        out = sc.conv_with_bias(self.kernel, self.bias, inp_features, nb.neighbors_index, kidx,
                                nb.neighbors_row_splits, inp_importance=inp_importance,
                                normalize=self.normalize)
        if self.activation:
            out = self.activation(out)
        return out


class SparseConvTranspose(SparseConv):
    """Open3D ``layers.SparseConvTranspose`` (sparseconvnet.py:447-482): the
    adjoint of SparseConv with the same filter indexing — output o receives
    input i with kernel index k exactly when SparseConv(out->in) would pair
    them; queries out_positions + offset*voxel_size, mirrored kernel index."""

    def forward(self, inp_features, inp_positions, out_positions, voxel_size, out_importance=None,
                fixed_radius_search_hash_table=None):
        if self.normalize:
            # each input's contribution divided by its number of output
            # neighbours (the inp_neighbors_* relation of ops.sparse_conv_transpose:
            # the same pairs grouped by input)
            nb, kidx = self._rulebook(inp_positions, out_positions, voxel_size, fixed_radius_search_hash_table,
                                      True, -1.0)
            n_in = inp_features.shape[0]
            cnt = torch.bincount(nb.neighbors_index.long(), minlength=n_in)
            irs = torch.zeros(n_in + 1, dtype=torch.int64, device=cnt.device)
            torch.cumsum(cnt, 0, out=irs[1:])
            out = sc.sparse_conv_transpose(self.kernel, out_importance, inp_features, None, None, irs,
                                           nb.neighbors_index, kidx, None, nb.neighbors_row_splits, normalize=True)
            if self.bias is not None:
                out = out + self.bias
            return self.activation(out) if self.activation else out
        out = self._lattice(inp_features, inp_positions, out_positions, voxel_size, fixed_radius_search_hash_table,
                            True, -1.0, bias=None, out_importance=out_importance)
        if out is not None:
            if self.bias is not None:
                out = out + self.bias
            return self.activation(out) if self.activation else out
        nb, kidx = self._rulebook(inp_positions, out_positions, voxel_size, fixed_radius_search_hash_table,
                                  True, -1.0)
        out = sc.sparse_conv_transpose(self.kernel, out_importance, inp_features, None, None, None,
                                       nb.neighbors_index, kidx, None, nb.neighbors_row_splits,
                                       normalize=False)
        if self.bias is not None:
            out = out + self.bias
        if self.activation:
            out = self.activation(out)
        return out
