// Packed weight-blob layouts shared by the kernels and the host packer
// (deepinteract_amd/packing.py mirrors these numbers; di_blob_bytes() exposes the totals).
//
// Matrix offsets are in packed blocks (16 output rows x 32 input features = 512 elements of
// the storage dtype; a 128x128 matrix = 32 blocks). Vector offsets are in fp32 elements
// (a 128-feature vector = 128 floats, packed [b][g][4]).
#pragma once

namespace di {

// ---- kind 0: node embedding + layer-0 Q/K/V (BN1 folded) --------------------------------
constexpr int EM_EMB = 0, EM_Q = 32, EM_K = 64, EM_V = 96, EM_NBLK = 128;
constexpr int EMV_Q = 0, EMV_K = 128, EMV_V = 256, EMV_N = 384;

// ---- kind 1: InitEdgeModule ----------------------------------------------------------------
// for t in {edge_messages, dist, dir, orient, amide}: geo0_t [8 blk] then c0_t [32 blk]; t = 0 holds
// only the collapsed combined_linear_0 . edge_messages_linear_0 map [8 blk] (blocks 8..39 zero)
constexpr int IE_T0 = 0;      // + 40*t
constexpr int IE_GEO1 = 200;  // 5 x [8 blk]
constexpr int IE_C1 = 240;    // combined_linear_1 (28 -> 32 rows) [2 x 4]
constexpr int IE_C2 = 248;    // combined_linear_2 (K 28 -> 32)    [8 x 1]
constexpr int IE_NBR = 256;   // layer-0 nbr_linear [8 x 4]
constexpr int IE_NBLK = 288;
// vectors: nbr_linear bias; with DI_GRAPH_GEO_REF the orientation terms as constants (kernel units):
// IEV_ORC = combined_linear_0's orientation slice . silu(orient_linear_0 (0,0,0,1)),
// IEV_OGATE = silu(orient_linear_1 (0,0,0,1))
constexpr int IEV_NBR = 0, IEV_ORC = 128, IEV_OGATE = 256, IEV_N = 384;

// ---- kind 2/3: edge layer (conformation + attention scores [+ edge output]) --------------
// stage 0 = geometric gates + downward_proj (one 36-block stage), final gate rides with final_linear
constexpr int EL_S0 = 0;      // dist gate [8x1] 0-7, dir 8-11, orient 12-15, amide 16-19, then DOWN
constexpr int EL_DOWN = 20;   // [4 x 4]
constexpr int EL_UP = 36;     // [8 x 2]
constexpr int EL_OM = 52;     // orig_msg_linear
constexpr int EL_RES = 84;    // 12 x [8x4]: pre0 l0..l2, pre1, post0, post1
constexpr int EL_RC = 468;
constexpr int EL_F = 500;     // final_linear [8x4]
constexpr int EL_FG = 532;    // final gate (sum of the 4 final_* geometric linears) [8x1]
constexpr int EL_P = 540;     // edge_feats_projection . BN1e
constexpr int EL_NBLK_FINAL = 572;
constexpr int EL_NBLK_CONF = 540;  // kind 6: conformation module alone (stages S0 .. final_linear)
constexpr int EL_OE = 572;
constexpr int EL_F1 = 604;    // 2 x [8x4] (hidden halves)
constexpr int EL_F2 = 668;    // 2 x [8x4] (input halves)
constexpr int EL_NN = 732;    // next layer's nbr_linear
constexpr int EL_NBLK = 764;
constexpr int ELV_OM = 0, ELV_RES = 128, ELV_RC = 1664, ELV_F = 1792, ELV_P = 1920;
constexpr int ELV_N_FINAL = 2048;
constexpr int ELV_N_CONF = 1920;
constexpr int ELV_OE = 2048, ELV_F1 = 2176, ELV_NN = 2432, ELV_N = 2560;

// ---- kind 4/5: node layer (aggregation + O_node + FFN [+ next Q/K/V]) ----------------------
constexpr int NL_ON = 0, NL_F1 = 32, NL_F2 = 96, NL_NBLK_FINAL = 160;
constexpr int NL_Q = 160, NL_NBLK = 256;
constexpr int NLV_ON = 0, NLV_F1 = 128, NLV_N_FINAL = 384;
constexpr int NLV_Q = 384, NLV_N = 768;

constexpr int POS_TABLE_ROWS = 2304;  // NODE_COUNT_LIMIT

}  // namespace di
