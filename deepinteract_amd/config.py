"""Model / graph constants for the GeoT hot path.

Names follow the reference's CLI flags and constants:
  --knn 20, --num_gnn_layers 2, --num_gnn_hidden_channels 128, --num_gnn_attention_heads 4,
  --num_interact_layers 14, --num_interact_hidden_channels 128
  (deepinteract_utils.py:1012-1019, deepinteract_modules.py:2200-2236),
  NODE_COUNT_LIMIT=2304, RESIDUE_COUNT_LIMIT=256, KNN=20 (deepinteract_constants.py:9-13),
  FEATURE_INDICES (deepinteract_constants.py:99-116), geo_nbrhd_size=2 (lit_model_predict.py:156).
"""
from dataclasses import dataclass

NODE_COUNT_LIMIT = 2304
RESIDUE_COUNT_LIMIT = 256
KNN = 20
GEO_NBRHD_SIZE = 2
NUM_RBF = 18
NUM_NODE_FEATS = 113
NUM_EDGE_FEATS = 28  # 'num_edge_features = 27' in lit_model_predict.py:138 is an off-by-one label
NUM_DIPS_FEATS = 106

FEATURE_INDICES = {
    'node_pos_enc': 0,
    'node_geo_feats_start': 1,
    'node_geo_feats_end': 7,
    'node_dips_plus_feats_start': 7,
    'node_dips_plus_feats_end': 113,
    'edge_pos_enc': 0,
    'edge_weights': 1,
    'edge_dist_feats_start': 2,
    'edge_dist_feats_end': 20,
    'edge_dir_feats_start': 20,
    'edge_dir_feats_end': 23,
    'edge_orient_feats_start': 23,
    'edge_orient_feats_end': 27,
    'edge_amide_angles': 27,
}


@dataclass(frozen=True)
class GeoTConfig:
    """Shape constants of DGLGeometricTransformer as LitGINI builds it
    (deepinteract_modules.py:1605-1622)."""
    num_node_input_feats: int = NUM_NODE_FEATS
    num_gnn_layers: int = 2
    num_gnn_hidden_channels: int = 128
    num_gnn_attention_heads: int = 4
    knn: int = KNN
    node_count_limit: int = NODE_COUNT_LIMIT
    shared_embed_size: int = 64
    geo_embed_size: int = 8  # dist/dir/orient/amide_embed_size
    num_pre_res_blocks: int = 2
    num_post_res_blocks: int = 2
    num_interact_layers: int = 14
    num_interact_hidden_channels: int = 128
    num_classes: int = 2
    bn_eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.num_gnn_hidden_channels // self.num_gnn_attention_heads
