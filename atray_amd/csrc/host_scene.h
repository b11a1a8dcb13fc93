// host_scene.h -- host-side scene types behind the opaque atr_mesh / atr_octree handles.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "engine.h"

namespace atr {

// ModelData (model.h:15-23), 0-based indices, 3 ints per face in each index array.
struct HostMesh {
    std::vector<V3> vertices, normals, texcoords;
    std::vector<int32_t> face_v, face_t, face_n;
    size_t nfaces() const { return face_v.size() / 3; }
};

// KD_Tree flattened in reference node order, plus parent/depth for the device traversal.
struct HostTree {
    int32_t nnodes = 0;
    std::vector<float> bounds;        // 6 per node
    std::vector<int32_t> children;    // children_start_position, 0 = leaf
    std::vector<int32_t> parent;      // -1 for the root
    std::vector<int32_t> depth;
    std::vector<uint32_t> leaf_first, leaf_count;
    std::vector<float> prim_vertices; // 9 per leaf primitive
    std::vector<uint32_t> prim_face;
};

// Leaf clusters: each leaf's primitives regrouped into spatial clusters of <= `size` (median
// splits on centroids), for the clustered leaf scan. Indices refer to the
// tree's leaf-ordered primitives (prim_face / prim_vertices).
struct LeafClusters {
    std::vector<uint32_t> order;  // cluster-ordered slot -> leaf-ordered primitive index
    std::vector<uint32_t> rank;   // slot -> rank of its primitive within its leaf
    std::vector<float> rec;       // 8 per cluster (DModel::clus)
    std::vector<float> normal;    // 3 per slot: ab x ac of its primitive
    std::vector<uint32_t> range;  // 2 per node: first cluster, cluster count (leaves only)
    float max_abs = 0.f;          // largest |coordinate| of any primitive vertex
};
int leaf_clusters(const HostTree& T, int size, LeafClusters& C);

// Inner-node table for the derived-box traversal: 3 float4 per inner node, in
// reference node order (inner id = rank among inner nodes). Fails with ATR_E_TREE_LAYOUT unless
// every inner node's 8 children boxes are the (lo|v, v|hi) combinations of its box and split
// point, bit for bit, as build_oct_kd_tree makes them (kd_tree.cpp:116-148). leaf_rank[node] =
// the leaf's rank in the static discovery order (-1 for inner nodes): leaf ids on the device.
int inner_table(const HostTree& T, std::vector<float4_t>& out, std::vector<int32_t>& leaf_rank);

// The device tables of one octree model (atr_scene_upload), built on the host: every array the
// kernels index, in the layouts of DESIGN.md §3. Kept apart from the upload so the sanitizer
// harness (tests/c/host_sanitize.cpp) checks the packing's sizes and index ranges.
struct PackedTree {
    std::vector<DNode> nodes;          // reference node order (LANE)
    std::vector<uint32_t> leaf_range;  // 2 per leaf rank: first leaf-ordered primitive, count
    std::vector<float4_t> inner;       // inner_table, 3 per inner node
    int32_t ninner = 0;
    std::vector<DTri> tris;            // leaf-ordered primitives, ab / ac precomputed (model.h:77-78)
    std::vector<float4_t> t0, t1;      // LANE's SoA streams of `tris`
    std::vector<float> t2;
    std::vector<uint32_t> tface;
    size_t nclusters = 0;
    std::vector<uint32_t> clus;        // 4 x kClusterBlock u32 per cluster: {lo, P}{hi, q}, normal words
    std::vector<uint32_t> cl_range;    // 2 per leaf rank: first cluster, cluster count
    std::vector<float4_t> prim;        // 3 per slot (kMaxClusterSize slots per cluster): 48-B records
    int32_t max_depth = 0;
    bool near_ok = false;              // traverse_pass_near's register stack fits the tree
};
int pack_tree(const HostTree& T, int cluster_size, PackedTree& P);
DTri make_tri(const float* v9, uint32_t face);

// load_model_data (OBJ_loader.cpp:278-360) on `threads` newline-aligned chunks (obj_parse.cpp);
// the result does not depend on `threads`.
int parse_obj_text(const char* text, size_t len, HostMesh& m, int threads = 1);
void mesh_aabb(const HostMesh& m, float out[6]);
void mesh_translate(HostMesh& m, float box[6], V3 c);
int octree_build(const HostMesh& m, uint32_t max_faces, HostTree& T);
int octree_build_device(const HostMesh& m, uint32_t max_faces, int device, HostTree& T, float* ms_out);  // build.hip
int octree_finish(HostTree& T);
void octree_stats(const HostTree& T, int64_t s[7]);
void camera_set(atr_camera& cm, V3 eye, V3 facing, int32_t w, int32_t h, int32_t aa, uint32_t spp,
                int32_t bounces, float h_fov);
int32_t reference_tiles(int32_t W, int32_t H, int32_t threads, atr_tile* out, int32_t cap);
int32_t balance_shard_tiles(int32_t W, int32_t H, int32_t side, int32_t world, const int64_t* costs,
                            int64_t rank0_extra, int32_t* owner);
int32_t shard_tiles(int32_t W, int32_t H, int32_t side, int32_t rank, int32_t world, atr_tile* out,
                    int32_t cap);

}  // namespace atr

struct atr_mesh { atr::HostMesh m; };
struct atr_octree { atr::HostTree t; };
