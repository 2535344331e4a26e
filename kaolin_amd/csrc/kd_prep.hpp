// kd_prep.hpp -- prepare_vertices' per-face forward arithmetic, shared by
// kd_prepare_fwd (kd_prepare.hip) and the binning count of the from-vertices DIB-R forward
// (kd_bin_count PREP, kd_binning.hip), so both produce the same bits.
//
// Reference: kaolin/render/mesh/utils.py:128-175 (prepare_vertices):
//   vertices_camera = pad(vertices, 1) @ camera_transform                 (utils.py:164-167)
//   vertices_image  = perspective_camera(vertices_camera, camera_proj)    (legacy.py:120-139)
//   face_vertices_* = index_vertices_by_faces(..., faces)                 (ops/mesh/mesh.py:24-45)
//   face_normals    = cross(v1 - v0, v2 - v0) / (|.| + 1e-10)             (trianglemesh.py:313-336)
#pragma once

#include "kd_common.hpp"

namespace kd {

template <typename T>
struct PrepArgs {
  int B, Bv;        // views; vertex batches (1 = shared by all views, else B)
  int64_t V, F;
  const T *vertices;   // (Bv, V, 3)
  const int64_t *faces;  // (F, 3)
  const T *proj;       // (3)
  const T *tf;         // (B, 4, 3)
};

// prepare_vertices' outputs written by the from-vertices binning count (nullptr fields: none)
template <typename T>
struct PrepOut {
  PrepArgs<T> a;  // a.vertices == nullptr: no prepare in the binning
  T *fvc;         // (B, F, 3, 3)
  T *fvi;         // (B, F, 3, 2)
  T *nrm;         // (B, F, 3)
};

template <typename T>
__device__ __forceinline__ void cam_point(const T *tf, const T *p, T c[3]) {
#pragma unroll
  for (int j = 0; j < 3; ++j) c[j] = p[0] * tf[j] + p[1] * tf[3 + j] + p[2] * tf[6 + j] + tf[9 + j];
}

// Face f of view b: camera-space corners c, image corners fi (x, y per corner) and the unit
// normal n, exactly as the reference composition rounds them.  (A caller whose workgroup holds
// one view passes it as b: no 64-bit division, and the view's transform is a uniform load.)
template <typename T>
__device__ __forceinline__ void prep_face_bf(const PrepArgs<T> &a, int b, int64_t f, T c[3][3],
                                             T fi[6], T n[3]) {
  const T *vb = a.vertices + (a.Bv == 1 ? 0 : (int64_t)b * a.V * 3);
  const T *tf = a.tf + (int64_t)b * 12;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int64_t v = a.faces[f * 3 + k];
    cam_point<T>(tf, vb + v * 3, c[k]);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const T pz = c[k][2] * a.proj[2];
    fi[k * 2 + 0] = c[k][0] * a.proj[0] / pz;
    fi[k * 2 + 1] = c[k][1] * a.proj[1] / pz;
  }
  const T e1[3] = {c[1][0] - c[0][0], c[1][1] - c[0][1], c[1][2] - c[0][2]};
  const T e2[3] = {c[2][0] - c[0][0], c[2][1] - c[0][1], c[2][2] - c[0][2]};
  const T r[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                  e1[0] * e2[1] - e1[1] * e2[0]};
  const T len = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]) + (T)1e-10;
  n[0] = r[0] / len;
  n[1] = r[1] / len;
  n[2] = r[2] / len;
}

// Face row i (view i / F).
template <typename T>
__device__ __forceinline__ void prep_face(const PrepArgs<T> &a, int64_t i, T c[3][3], T fi[6],
                                          T n[3]) {
  const int b = (int)(i / a.F);
  prep_face_bf<T>(a, b, i - (int64_t)b * a.F, c, fi, n);
}

// Copies n elements of T from LDS to global memory with the workgroup, 16-byte vectors when
// both sides allow (the rows of a workgroup are contiguous in every output).
template <typename T>
__device__ __forceinline__ void lds_to_global(T *dst, const T *src, int n) {
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0 && (n * sizeof(T)) % 16 == 0) {
    const int nv = n * (int)sizeof(T) / 16;
    for (int k = threadIdx.x; k < nv; k += kBlock)
      reinterpret_cast<float4 *>(dst)[k] = reinterpret_cast<const float4 *>(src)[k];
  } else {
    for (int k = threadIdx.x; k < n; k += kBlock) dst[k] = src[k];
  }
}

// Stages face row (thread) outputs into LDS rows of 9 / 6 / 3 values.
template <typename T>
__device__ __forceinline__ void prep_stage(const T c[3][3], const T fi[6], const T n[3], T *s_c,
                                           T *s_i, T *s_n) {
  T *oc = s_c + threadIdx.x * 9;
  T *oi = s_i + threadIdx.x * 6;
  T *on = s_n + threadIdx.x * 3;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    oc[k * 3 + 0] = c[k][0];
    oc[k * 3 + 1] = c[k][1];
    oc[k * 3 + 2] = c[k][2];
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) oi[k] = fi[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) on[k] = n[k];
}

}  // namespace kd
