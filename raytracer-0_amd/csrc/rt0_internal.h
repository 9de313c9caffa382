// rt0_internal.h -- declarations shared by the host-side translation units.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt0.h"

struct BvhNode;
struct TriDev;

namespace rt0h {
int lookup_material(const std::string &name, rt0_mesh &m);
int parse_scene_glsl(const char *text, const char *const *sdf, int n_sdf, std::vector<rt0_mesh> &meshes,
                     int &n_euclid, int &n_sdfs, int &n_models, std::vector<int32_t> &lights, std::string &err);
// OBJ text -> positions (3 floats each) + triangles (3 indices each); polygons
// are fan-triangulated, negative (relative) indices resolved
int parse_obj(const char *text, size_t len, std::vector<float> &pos, std::vector<int32_t> &tris, std::string &err);
void default_config(rt0_config &c);
// binned-SAH BVH (rt0_bvh_sah.cpp) of n triangles (v: 9 floats each, model:
// owner tags with RT0_TRI_CULL_BIT) -> pre-order inner nodes + leaf-order
// triangles; returns the depth (edges root -> deepest leaf), -1 for n <= 0
int bvh_build_sah(int n, const float *v, const int32_t *model, std::vector<BvhNode> &nodes, std::vector<TriDev> &tris);
// renumber the tree so that every node of its top levels comes first,
// breadth-first (at most max_nodes of them, whole levels), the rest after in
// their pre-order; returns how many lead (the LDS treelet, bvh_fetch)
int bvh_treelet_order(std::vector<BvhNode> &nodes, int max_nodes);
int parse_config(const char *const *defines, int nd, const char *const *constants, int nc, rt0_config &c,
                 std::string &err);
}  // namespace rt0h
