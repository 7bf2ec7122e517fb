// mesh_unstructured.cpp -- unstructured tetrahedral / hexahedral meshes for the PCSHELL
// (SURVEY.md §8f row f3): Gmsh reader, cell and face geometry, the exact mesh -> Cartesian
// intersection ("crude") matrix, the upwind transport operator over the mesh faces, and the
// implicit GMRES time loop with the remapped circulant FFT preconditioner.
//
//   cfp_mesh_read_gmsh / cfp_mesh_create   SOLVERLAB Mesh(filename) (tests/...impl_mpi.cxx:250)
//   cfp_mesh_min_ratio_vol_surf            Mesh::minRatioVolSurf (tests/...impl_mpi.cxx:51)
//   cfp_mesh_crude_matrix_cartesian        MEDCoupling getCrudeMatrix, P0->P0 (ToDo.md:12)
//   MatCreateMeshCartesianRemap            intersectionMatrix (src/PCSHELLFft_3D.hxx:17)
//   getFFTPrec3DContextMesh                getFFTPrec3DContext(..., Mesh) (:101-151)
//   cfp_mesh_transport_csr                 computeDivergenceMatrix (src/TransportEquation.cxx:75-133)
//   initial_conditions_shock_mesh          initial_conditions_shock (:25-73)
//   TransportEquationGMRESMesh             TransportEquation_impl_mpi on Mesh(filename)
//
// Host-side set-up only (as MatSetValue assembly and MEDCoupling are in the reference).
#ifndef CFP_WITH_PETSC
#include <sys/time.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/circulant_fft.h"
#include "../../include/mesh_unstructured.h"
#include "cfp_host.h"

using cfp::set_error;

namespace {

typedef std::array<double, 3> P3;
typedef std::array<P3, 4> Tet;

P3 sub(const P3& a, const P3& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
P3 cross(const P3& a, const P3& b) {
  return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}
double dot(const P3& a, const P3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
double tet_vol(const Tet& t) { return std::fabs(dot(sub(t[1], t[0]), cross(sub(t[2], t[0]), sub(t[3], t[0])))) / 6.0; }

// Gmsh node orderings: tet 0-3; hex 0-3 bottom (counter-clockwise), 4-7 above them.
const int kTetFaces[4][3] = {{0, 1, 2}, {0, 1, 3}, {0, 2, 3}, {1, 2, 3}};
const int kHexFaces[6][4] = {{0, 3, 2, 1}, {0, 1, 5, 4}, {0, 4, 7, 3}, {1, 2, 6, 5}, {2, 3, 7, 6}, {4, 5, 6, 7}};
// six tetrahedra around the 0-6 diagonal (exact for a convex hexahedron)
const int kHexTets[6][4] = {{0, 1, 2, 6}, {0, 2, 3, 6}, {0, 3, 7, 6}, {0, 7, 4, 6}, {0, 4, 5, 6}, {0, 5, 1, 6}};

struct FaceKey {
  int64_t v[4];
  bool operator==(const FaceKey& o) const { return std::memcmp(v, o.v, sizeof(v)) == 0; }
};
struct FaceKeyHash {
  size_t operator()(const FaceKey& k) const {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 4; ++i) h = (h ^ (uint64_t)k.v[i]) * 1099511628211ull;
    return (size_t)h;
  }
};

// v (d <= 0 side) clipped against the plane d = 0: a' = a + t (b - a), t = da / (da - db)
P3 cut(const P3& a, const P3& b, double da, double db) {
  const double t = da / (da - db);
  return {a[0] + t * (b[0] - a[0]), a[1] + t * (b[1] - a[1]), a[2] + t * (b[2] - a[2])};
}

// Keep the part of tet t with s * (p[axis] - c) <= 0; appends 0-3 tetrahedra to out.
void clip_tet(const Tet& t, int axis, double c, double s, std::vector<Tet>& out) {
  double d[4];
  int in[4], ou[4], ni = 0, no = 0;
  for (int i = 0; i < 4; ++i) {
    d[i] = s * (t[i][axis] - c);
    if (d[i] <= 0) in[ni++] = i;
    else ou[no++] = i;
  }
  if (ni == 4) { out.push_back(t); return; }
  if (ni == 0) return;
  if (ni == 1) {
    const int A = in[0];
    Tet r = {t[A], cut(t[A], t[ou[0]], d[A], d[ou[0]]), cut(t[A], t[ou[1]], d[A], d[ou[1]]),
             cut(t[A], t[ou[2]], d[A], d[ou[2]])};
    out.push_back(r);
    return;
  }
  // prism (P0 P1 P2)-(Q0 Q1 Q2) with lateral edges Pi-Qi -> 3 tetrahedra
  auto prism = [&](const P3& P0, const P3& P1, const P3& P2, const P3& Q0, const P3& Q1, const P3& Q2) {
    out.push_back({P0, P1, P2, Q2});
    out.push_back({P0, P1, Q2, Q1});
    out.push_back({P0, Q1, Q2, Q0});
  };
  if (ni == 3) {  // the tet minus the corner at the outside vertex D
    const int A = in[0], B = in[1], C = in[2], D = ou[0];
    prism(t[A], t[B], t[C], cut(t[A], t[D], d[A], d[D]), cut(t[B], t[D], d[B], d[D]), cut(t[C], t[D], d[C], d[D]));
    return;
  }
  // ni == 2: A, B inside, C, D outside; triangles (A, AC, AD) and (B, BC, BD)
  const int A = in[0], B = in[1], C = ou[0], D = ou[1];
  prism(t[A], cut(t[A], t[C], d[A], d[C]), cut(t[A], t[D], d[A], d[D]), t[B], cut(t[B], t[C], d[B], d[C]),
        cut(t[B], t[D], d[B], d[D]));
}

// keep lo <= p[axis] <= hi
void clip_slab(const std::vector<Tet>& in, int axis, double lo, double hi, std::vector<Tet>& out) {
  std::vector<Tet> tmp;
  out.clear();
  for (const Tet& t : in) {
    tmp.clear();
    clip_tet(t, axis, hi, 1.0, tmp);
    for (const Tet& u : tmp) clip_tet(u, axis, lo, -1.0, out);
  }
}

void tets_range(const std::vector<Tet>& ts, int axis, double& lo, double& hi) {
  lo = 1e300;
  hi = -1e300;
  for (const Tet& t : ts)
    for (int i = 0; i < 4; ++i) {
      lo = std::min(lo, t[i][axis]);
      hi = std::max(hi, t[i][axis]);
    }
}

double wall() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
}

}  // namespace

struct cfp_mesh_s {
  std::vector<double> xyz;  // 3 per node
  std::vector<int64_t> cptr, cnodes;
  std::vector<double> vol, ctr;  // per cell: measure, barycentre (3)
  std::vector<int64_t> f0, f1;   // per face: cells (f1 = -1 on the border)
  std::vector<double> farea, fnormal;  // per face: measure, unit normal out of f0 (3)
  std::vector<int64_t> cfptr, cfaces;  // cell -> its faces
  double bbox[6];
  // last crude matrix (the two-call protocol computes it once)
  int64_t cm_n[3] = {0, 0, 0};
  double cm_box[6] = {0, 0, 0, 0, 0, 0};
  std::vector<int64_t> cm_rowptr, cm_col;
  std::vector<double> cm_val;

  P3 node(int64_t i) const { return {xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]}; }
  int64_t ncells() const { return (int64_t)cptr.size() - 1; }
  void cell_tets(int64_t c, std::vector<Tet>& out) const {
    out.clear();
    const int64_t* v = &cnodes[(size_t)cptr[c]];
    if (cptr[c + 1] - cptr[c] == 4) {
      out.push_back({node(v[0]), node(v[1]), node(v[2]), node(v[3])});
    } else {
      for (auto& q : kHexTets) out.push_back({node(v[q[0]]), node(v[q[1]]), node(v[q[2]]), node(v[q[3]])});
    }
  }
  int build();
};

int cfp_mesh_s::build() {
  const int64_t nn = (int64_t)xyz.size() / 3, nc = ncells();
  if (nc < 1) return set_error(CFP_ERR_ARG_SIZ, "mesh has no 3-D cells");
  for (int d = 0; d < 3; ++d) {
    bbox[2 * d] = 1e300;
    bbox[2 * d + 1] = -1e300;
  }
  for (int64_t i = 0; i < nn; ++i)
    for (int d = 0; d < 3; ++d) {
      bbox[2 * d] = std::min(bbox[2 * d], xyz[3 * i + d]);
      bbox[2 * d + 1] = std::max(bbox[2 * d + 1], xyz[3 * i + d]);
    }
  vol.assign((size_t)nc, 0.0);
  ctr.assign((size_t)(3 * nc), 0.0);
  std::vector<Tet> ts;
  for (int64_t c = 0; c < nc; ++c) {
    const int64_t k = cptr[c + 1] - cptr[c];
    if (k != 4 && k != 8) return set_error(CFP_ERR_SUP, "cell %lld has %lld nodes (4 or 8 supported)", (long long)c, (long long)k);
    for (int64_t p = cptr[c]; p < cptr[c + 1]; ++p)
      if (cnodes[(size_t)p] < 0 || cnodes[(size_t)p] >= nn)
        return set_error(CFP_ERR_ARG_OUTOFRANGE, "cell %lld references node %lld", (long long)c, (long long)cnodes[(size_t)p]);
    cell_tets(c, ts);
    double v = 0, g[3] = {0, 0, 0};
    for (const Tet& t : ts) {
      const double w = tet_vol(t);
      v += w;
      for (int d = 0; d < 3; ++d) g[d] += w * 0.25 * (t[0][d] + t[1][d] + t[2][d] + t[3][d]);
    }
    if (!(v > 0)) return set_error(CFP_ERR_ARG_WRONG, "cell %lld has zero volume", (long long)c);
    vol[(size_t)c] = v;
    for (int d = 0; d < 3; ++d) ctr[(size_t)(3 * c + d)] = g[d] / v;
  }
  // faces: shared by sorted node keys
  std::unordered_map<FaceKey, int64_t, FaceKeyHash> map;
  map.reserve((size_t)(4 * nc));
  cfptr.assign((size_t)nc + 1, 0);
  cfaces.clear();
  for (int64_t c = 0; c < nc; ++c) {
    const int64_t* v = &cnodes[(size_t)cptr[c]];
    const bool tet = cptr[c + 1] - cptr[c] == 4;
    const int nf = tet ? 4 : 6, nv = tet ? 3 : 4;
    const P3 cc = {ctr[(size_t)(3 * c)], ctr[(size_t)(3 * c + 1)], ctr[(size_t)(3 * c + 2)]};
    for (int f = 0; f < nf; ++f) {
      int64_t fv[4];
      for (int i = 0; i < nv; ++i) fv[i] = v[tet ? kTetFaces[f][i] : kHexFaces[f][i]];
      FaceKey key;
      for (int i = 0; i < 4; ++i) key.v[i] = i < nv ? fv[i] : -1;
      std::sort(key.v, key.v + nv);
      auto it = map.find(key);
      if (it != map.end()) {
        const int64_t id = it->second;
        if (f1[(size_t)id] >= 0)
          return set_error(CFP_ERR_ARG_WRONG, "face shared by more than two cells (cell %lld)", (long long)c);
        f1[(size_t)id] = c;
        cfaces.push_back(id);
        continue;
      }
      // area vector from this cell's ordering, turned to point out of the cell
      P3 A, fc = {0, 0, 0};
      if (nv == 3) {
        A = cross(sub(node(fv[1]), node(fv[0])), sub(node(fv[2]), node(fv[0])));
      } else {
        A = cross(sub(node(fv[2]), node(fv[0])), sub(node(fv[3]), node(fv[1])));
      }
      for (int i = 0; i < nv; ++i)
        for (int d = 0; d < 3; ++d) fc[d] += node(fv[i])[d] / nv;
      if (dot(A, sub(fc, cc)) < 0)
        for (int d = 0; d < 3; ++d) A[d] = -A[d];
      const double m = std::sqrt(dot(A, A));
      if (!(m > 0)) return set_error(CFP_ERR_ARG_WRONG, "degenerate face in cell %lld", (long long)c);
      const int64_t id = (int64_t)f0.size();
      map.emplace(key, id);
      f0.push_back(c);
      f1.push_back(-1);
      farea.push_back(0.5 * m);
      for (int d = 0; d < 3; ++d) fnormal.push_back(A[d] / m);
      cfaces.push_back(id);
    }
    cfptr[(size_t)c + 1] = (int64_t)cfaces.size();
  }
  return CFP_SUCCESS;
}

extern "C" int cfp_mesh_create(int64_t nnodes, const double* xyz, int64_t ncells, const int64_t* cell_ptr,
                               const int64_t* cell_nodes, cfp_mesh_t* mesh) {
  if (!mesh || !xyz || !cell_ptr || !cell_nodes) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *mesh = nullptr;
  if (nnodes < 4 || ncells < 1) return set_error(CFP_ERR_ARG_SIZ, "mesh needs >= 4 nodes and >= 1 cell");
  cfp_mesh_s* m = new cfp_mesh_s;
  m->xyz.assign(xyz, xyz + 3 * nnodes);
  m->cptr.assign(cell_ptr, cell_ptr + ncells + 1);
  if (m->cptr[0] != 0) {
    delete m;
    return set_error(CFP_ERR_ARG_WRONG, "cell_ptr[0] must be 0");
  }
  m->cnodes.assign(cell_nodes, cell_nodes + cell_ptr[ncells]);
  const int rc = m->build();
  if (rc) {
    delete m;
    return rc;
  }
  *mesh = m;
  return CFP_SUCCESS;
}

// Gmsh ASCII 2.x ($Nodes: id x y z; $Elements: id type ntags tags... nodes...) and 4.1
// (entity blocks: $Nodes "dim tag parametric n" then n tags then n coordinate lines;
// $Elements "dim tag type n" then n lines "id nodes...").
extern "C" int cfp_mesh_read_gmsh(const char* path, cfp_mesh_t* mesh) {
  if (!path || !mesh) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  *mesh = nullptr;
  std::ifstream in(path);
  if (!in) return set_error(CFP_ERR_ARG_WRONG, "cannot open %s", path);
  std::string tok;
  std::unordered_map<int64_t, int64_t> id2idx;
  std::vector<double> xyz;
  std::vector<int64_t> cptr(1, 0), cnodes;
  double ver = 0;
  auto keep = [&](int64_t type, const int64_t* nodes) -> bool {
    const int nv = type == 4 ? 4 : 8;
    for (int i = 0; i < nv; ++i) {
      auto it = id2idx.find(nodes[i]);
      if (it == id2idx.end()) return false;
      cnodes.push_back(it->second);
    }
    cptr.push_back((int64_t)cnodes.size());
    return true;
  };
  auto nverts = [](int64_t type) -> int {  // nodes per element of the Gmsh types we may meet
    switch (type) {
      case 1: return 2;  case 2: return 3;  case 3: return 4;  case 4: return 4;
      case 5: return 8;  case 6: return 6;  case 7: return 5;  case 15: return 1;
      default: return -1;
    }
  };
  while (in >> tok) {
    if (tok == "$MeshFormat") {
      int ftype = -1, dsize = 0;
      in >> ver >> ftype >> dsize;
      if (!((ver >= 2.0 && ver < 3.0) || (ver >= 4.0 && ver < 5.0)) || ftype != 0)
        return set_error(CFP_ERR_SUP, "%s: Gmsh format %g type %d (ASCII 2.x or 4.1 supported)", path, ver, ftype);
    } else if (tok == "$Nodes") {
      if (ver >= 4.0) {
        int64_t nblocks, nnodes, mn, mx;
        in >> nblocks >> nnodes >> mn >> mx;
        for (int64_t b = 0; b < nblocks; ++b) {
          int64_t dim, tag, param, n;
          in >> dim >> tag >> param >> n;
          if (param) return set_error(CFP_ERR_SUP, "%s: parametric nodes unsupported", path);
          std::vector<int64_t> ids((size_t)n);
          for (auto& id : ids) in >> id;
          for (int64_t i = 0; i < n; ++i) {
            double x, y, z;
            in >> x >> y >> z;
            id2idx[ids[(size_t)i]] = (int64_t)xyz.size() / 3;
            xyz.push_back(x);
            xyz.push_back(y);
            xyz.push_back(z);
          }
        }
      } else {
        int64_t n;
        in >> n;
        for (int64_t i = 0; i < n; ++i) {
          int64_t id;
          double x, y, z;
          in >> id >> x >> y >> z;
          id2idx[id] = i;
          xyz.push_back(x);
          xyz.push_back(y);
          xyz.push_back(z);
        }
      }
      if (!in) return set_error(CFP_ERR_ARG_WRONG, "%s: truncated $Nodes", path);
    } else if (tok == "$Elements") {
      int64_t nodes[8];
      if (ver >= 4.0) {
        int64_t nblocks, nel, mn, mx;
        in >> nblocks >> nel >> mn >> mx;
        for (int64_t b = 0; b < nblocks; ++b) {
          int64_t dim, tag, type, n;
          in >> dim >> tag >> type >> n;
          const int nv = nverts(type);
          if (nv < 0) return set_error(CFP_ERR_SUP, "%s: element type %lld", path, (long long)type);
          for (int64_t e = 0; e < n; ++e) {
            int64_t id, skip;
            in >> id;
            for (int i = 0; i < nv; ++i) {
              if (type == 4 || type == 5) in >> nodes[i];
              else in >> skip;
            }
            if ((type == 4 || type == 5) && !keep(type, nodes))
              return set_error(CFP_ERR_ARG_WRONG, "%s: element %lld uses an unknown node", path, (long long)id);
          }
        }
      } else {
        int64_t n;
        in >> n;
        for (int64_t e = 0; e < n; ++e) {
          int64_t id, type, ntags, skip;
          in >> id >> type >> ntags;
          for (int64_t t = 0; t < ntags; ++t) in >> skip;
          const int nv = nverts(type);
          if (nv < 0) return set_error(CFP_ERR_SUP, "%s: element type %lld", path, (long long)type);
          for (int i = 0; i < nv; ++i) {
            if (type == 4 || type == 5) in >> nodes[i];
            else in >> skip;
          }
          if ((type == 4 || type == 5) && !keep(type, nodes))
            return set_error(CFP_ERR_ARG_WRONG, "%s: element %lld uses an unknown node", path, (long long)id);
        }
      }
      if (!in) return set_error(CFP_ERR_ARG_WRONG, "%s: truncated $Elements", path);
    }
  }
  if (ver == 0) return set_error(CFP_ERR_ARG_WRONG, "%s: no $MeshFormat section", path);
  if (cptr.size() < 2) return set_error(CFP_ERR_ARG_SIZ, "%s: no tetrahedra or hexahedra", path);
  // merge nodes with identical coordinates (some FVCA files, e.g. the Kershaw tetrahedra,
  // repeat the nodes of internal surfaces; the cells would not be connected through them)
  {
    const int64_t nn = (int64_t)xyz.size() / 3;
    std::vector<int64_t> order((size_t)nn), remap((size_t)nn);
    for (int64_t i = 0; i < nn; ++i) order[(size_t)i] = i;
    auto lt = [&](int64_t a, int64_t b) {
      for (int d = 0; d < 3; ++d)
        if (xyz[3 * a + d] != xyz[3 * b + d]) return xyz[3 * a + d] < xyz[3 * b + d];
      return a < b;
    };
    std::sort(order.begin(), order.end(), lt);
    std::vector<double> merged;
    merged.reserve(xyz.size());
    for (size_t k = 0; k < order.size(); ++k) {
      const int64_t i = order[k];
      const bool same = k > 0 && xyz[3 * i] == xyz[3 * order[k - 1]] && xyz[3 * i + 1] == xyz[3 * order[k - 1] + 1] &&
                        xyz[3 * i + 2] == xyz[3 * order[k - 1] + 2];
      if (!same) {
        merged.push_back(xyz[3 * i]);
        merged.push_back(xyz[3 * i + 1]);
        merged.push_back(xyz[3 * i + 2]);
      }
      remap[(size_t)i] = (int64_t)merged.size() / 3 - 1;
    }
    if ((int64_t)merged.size() / 3 != nn) {
      for (auto& v : cnodes) v = remap[(size_t)v];
      xyz.swap(merged);
    }
  }
  return cfp_mesh_create((int64_t)xyz.size() / 3, xyz.data(), (int64_t)cptr.size() - 1, cptr.data(), cnodes.data(),
                         mesh);
}

extern "C" int cfp_mesh_destroy(cfp_mesh_t mesh) {
  delete mesh;
  return CFP_SUCCESS;
}

extern "C" int cfp_mesh_info(cfp_mesh_t m, int64_t* nnodes, int64_t* ncells, int64_t* nfaces, double bbox[6]) {
  if (!m) return set_error(CFP_ERR_ARG_NULL, "NULL mesh");
  if (nnodes) *nnodes = (int64_t)m->xyz.size() / 3;
  if (ncells) *ncells = m->ncells();
  if (nfaces) *nfaces = (int64_t)m->f0.size();
  if (bbox) std::memcpy(bbox, m->bbox, sizeof(m->bbox));
  return CFP_SUCCESS;
}

extern "C" int cfp_mesh_cell_geometry(cfp_mesh_t m, double* volumes, double* centers) {
  if (!m) return set_error(CFP_ERR_ARG_NULL, "NULL mesh");
  if (volumes) std::memcpy(volumes, m->vol.data(), sizeof(double) * m->vol.size());
  if (centers) std::memcpy(centers, m->ctr.data(), sizeof(double) * m->ctr.size());
  return CFP_SUCCESS;
}

extern "C" int cfp_mesh_faces(cfp_mesh_t m, int64_t* cell0, int64_t* cell1, double* measure, double* normal) {
  if (!m) return set_error(CFP_ERR_ARG_NULL, "NULL mesh");
  if (cell0) std::memcpy(cell0, m->f0.data(), sizeof(int64_t) * m->f0.size());
  if (cell1) std::memcpy(cell1, m->f1.data(), sizeof(int64_t) * m->f1.size());
  if (measure) std::memcpy(measure, m->farea.data(), sizeof(double) * m->farea.size());
  if (normal) std::memcpy(normal, m->fnormal.data(), sizeof(double) * m->fnormal.size());
  return CFP_SUCCESS;
}

extern "C" int cfp_mesh_min_ratio_vol_surf(cfp_mesh_t m, double* ratio) {
  if (!m || !ratio) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  double r = 1e300;
  for (int64_t c = 0; c < m->ncells(); ++c) {
    double s = 0;
    for (int64_t p = m->cfptr[(size_t)c]; p < m->cfptr[(size_t)c + 1]; ++p) s += m->farea[(size_t)m->cfaces[(size_t)p]];
    r = std::min(r, m->vol[(size_t)c] / s);
  }
  *ratio = r;
  return CFP_SUCCESS;
}

// Intersection volumes of every mesh cell with the Cartesian cells: each tetrahedron of the
// cell is clipped to the x slab of each Cartesian column it spans, the pieces to the y slabs,
// then to the z slabs; the pieces' volumes are the entries.  Entries below 1e-14 |C| (pieces
// that only touch a grid plane) are dropped.
static int crude_build(cfp_mesh_s* m, int64_t nx, int64_t ny, int64_t nz, const double* box) {
  const int64_t n[3] = {nx, ny, nz};
  if (m->cm_n[0] == nx && m->cm_n[1] == ny && m->cm_n[2] == nz && std::memcmp(m->cm_box, box, sizeof(m->cm_box)) == 0)
    return CFP_SUCCESS;
  double h[3];
  for (int d = 0; d < 3; ++d) h[d] = (box[2 * d + 1] - box[2 * d]) / (double)n[d];
  struct Ent {
    int64_t row, col;
    double v;
  };
  std::vector<Ent> ent;
  std::vector<Tet> ts, px, py, pz;
  auto cell_range = [&](const std::vector<Tet>& t, int d, int64_t& i0, int64_t& i1) {
    double lo, hi;
    tets_range(t, d, lo, hi);
    i0 = std::max<int64_t>(0, (int64_t)std::floor((lo - box[2 * d]) / h[d]));
    i1 = std::min<int64_t>(n[d] - 1, (int64_t)std::floor((hi - box[2 * d]) / h[d]));
  };
  for (int64_t c = 0; c < m->ncells(); ++c) {
    m->cell_tets(c, ts);
    const double tiny = 1e-14 * m->vol[(size_t)c];
    int64_t x0, x1;
    cell_range(ts, 0, x0, x1);
    for (int64_t ix = x0; ix <= x1; ++ix) {
      clip_slab(ts, 0, box[0] + ix * h[0], box[0] + (ix + 1) * h[0], px);
      if (px.empty()) continue;
      int64_t y0, y1;
      cell_range(px, 1, y0, y1);
      for (int64_t iy = y0; iy <= y1; ++iy) {
        clip_slab(px, 1, box[2] + iy * h[1], box[2] + (iy + 1) * h[1], py);
        if (py.empty()) continue;
        int64_t z0, z1;
        cell_range(py, 2, z0, z1);
        for (int64_t iz = z0; iz <= z1; ++iz) {
          clip_slab(py, 2, box[4] + iz * h[2], box[4] + (iz + 1) * h[2], pz);
          double v = 0;
          for (const Tet& t : pz) v += tet_vol(t);
          if (v > tiny) ent.push_back({ix + nx * (iy + ny * iz), c, v});
        }
      }
    }
  }
  std::sort(ent.begin(), ent.end(), [](const Ent& a, const Ent& b) { return a.row != b.row ? a.row < b.row : a.col < b.col; });
  const int64_t N = nx * ny * nz;
  m->cm_rowptr.assign((size_t)N + 1, 0);
  m->cm_col.clear();
  m->cm_val.clear();
  for (size_t k = 0; k < ent.size(); ++k) {
    if (!m->cm_col.empty() && k > 0 && ent[k].row == ent[k - 1].row && ent[k].col == ent[k - 1].col) {
      m->cm_val.back() += ent[k].v;  // cannot happen (one entry per (cell, box)), kept for safety
      continue;
    }
    m->cm_col.push_back(ent[k].col);
    m->cm_val.push_back(ent[k].v);
    m->cm_rowptr[(size_t)ent[k].row + 1] += 1;
  }
  for (int64_t r = 0; r < N; ++r) m->cm_rowptr[(size_t)r + 1] += m->cm_rowptr[(size_t)r];
  m->cm_n[0] = nx;
  m->cm_n[1] = ny;
  m->cm_n[2] = nz;
  std::memcpy(m->cm_box, box, sizeof(m->cm_box));
  return CFP_SUCCESS;
}

extern "C" int cfp_mesh_crude_matrix_cartesian(cfp_mesh_t m, int64_t nx, int64_t ny, int64_t nz, const double bbox[6],
                                               int64_t* nnz, int64_t* rowptr, int64_t* col, double* val) {
  if (!m || !nnz) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (nx < 1 || ny < 1 || nz < 1) return set_error(CFP_ERR_ARG_OUTOFRANGE, "grid sizes must be >= 1");
  const double* box = bbox ? bbox : m->bbox;
  for (int d = 0; d < 3; ++d)
    if (!(box[2 * d + 1] > box[2 * d])) return set_error(CFP_ERR_ARG_OUTOFRANGE, "empty bounding box on axis %d", d);
  const int rc = crude_build(m, nx, ny, nz, box);
  if (rc) return rc;
  *nnz = (int64_t)m->cm_col.size();
  if (rowptr && col && val) {
    std::memcpy(rowptr, m->cm_rowptr.data(), sizeof(int64_t) * m->cm_rowptr.size());
    std::memcpy(col, m->cm_col.data(), sizeof(int64_t) * m->cm_col.size());
    std::memcpy(val, m->cm_val.data(), sizeof(double) * m->cm_val.size());
  }
  return CFP_SUCCESS;
}

// computeDivergenceMatrix, src/TransportEquation.cxx:75-133, over the faces of each cell
static void transport_rows(const cfp_mesh_s* m, double dt, const double a[3], int sign_mode, double shift,
                           std::vector<int64_t>& rowptr, std::vector<int64_t>& col, std::vector<double>& val) {
  const double sgn = sign_mode == CFP_UPWIND_REFERENCE ? -1.0 : 1.0;
  const int64_t nc = m->ncells();
  rowptr.assign((size_t)nc + 1, 0);
  col.clear();
  val.clear();
  std::vector<std::pair<int64_t, double>> row;
  for (int64_t j = 0; j < nc; ++j) {
    row.clear();
    double diag = shift;
    const double vj = m->vol[(size_t)j];
    for (int64_t p = m->cfptr[(size_t)j]; p < m->cfptr[(size_t)j + 1]; ++p) {
      const int64_t f = m->cfaces[(size_t)p];
      const int64_t other = m->f0[(size_t)f] == j ? m->f1[(size_t)f] : m->f0[(size_t)f];
      if (other < 0) continue;  // border: Neumann, nothing (:114-129)
      const double s = m->f0[(size_t)f] == j ? 1.0 : -1.0;  // normal out of cell j
      const double* nf = &m->fnormal[(size_t)(3 * f)];
      const double un = s * (nf[0] * a[0] + nf[1] * a[1] + nf[2] * a[2]);
      const double coef = dt * m->farea[(size_t)f] / vj;
      if (un > 0) diag += coef * un;                       // :109-110
      else row.push_back({other, sgn * coef * un});        // :111-112 (reference: -coef un)
    }
    row.push_back({j, diag});
    std::sort(row.begin(), row.end());
    size_t w = 0;  // merge repeated columns (two faces shared with one neighbour)
    for (size_t k = 0; k < row.size(); ++k) {
      if (w > 0 && row[w - 1].first == row[k].first) row[w - 1].second += row[k].second;
      else row[w++] = row[k];
    }
    for (size_t k = 0; k < w; ++k) {
      if (row[k].second == 0.0 && row[k].first != j) continue;
      col.push_back(row[k].first);
      val.push_back(row[k].second);
      val.push_back(0.0);
    }
    rowptr[(size_t)j + 1] = (int64_t)col.size();
  }
}

extern "C" int cfp_mesh_transport_csr(cfp_mesh_t m, double dt, const double a[3], int sign_mode, double shift,
                                      int64_t* nnz, int64_t* rowptr, int64_t* col, double* val) {
  if (!m || !a || !nnz) return set_error(CFP_ERR_ARG_NULL, "NULL argument");
  if (sign_mode != CFP_UPWIND_REFERENCE && sign_mode != CFP_UPWIND_FIXED)
    return set_error(CFP_ERR_ARG_OUTOFRANGE, "sign_mode must be CFP_UPWIND_REFERENCE or CFP_UPWIND_FIXED");
  std::vector<int64_t> rp, cl;
  std::vector<double> vl;
  transport_rows(m, dt, a, sign_mode, shift, rp, cl, vl);
  *nnz = (int64_t)cl.size();
  if (rowptr && col && val) {
    std::memcpy(rowptr, rp.data(), sizeof(int64_t) * rp.size());
    std::memcpy(col, cl.data(), sizeof(int64_t) * cl.size());
    std::memcpy(val, vl.data(), sizeof(double) * vl.size());
  }
  return CFP_SUCCESS;
}

// ------------------------------------------------------------------ PETSc-level entry points
extern "C" PetscErrorCode MatCreateMeshCartesianRemap(cfp_mesh_t m, PetscInt nx, PetscInt ny, PetscInt nz,
                                                      const PetscReal bbox[6], Mat* toCart, Mat* toMesh) {
  PetscFunctionBeginUser;
  PetscCheck(m, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "MatCreateMeshCartesianRemap: NULL mesh");
  int64_t nnz = 0;
  const int rc = cfp_mesh_crude_matrix_cartesian(m, nx, ny, nz, bbox, &nnz, nullptr, nullptr, nullptr);
  PetscCheck(rc == CFP_SUCCESS, PETSC_COMM_SELF, rc, cfp_last_error());
  const int64_t N = nx * ny * nz, nc = m->ncells();
  const std::vector<int64_t>& rp = m->cm_rowptr;
  const std::vector<int64_t>& cl = m->cm_col;
  const std::vector<double>& vl = m->cm_val;
  if (toCart) {
    std::vector<PetscScalar> a((size_t)nnz);
    for (int64_t r = 0; r < N; ++r) {
      double s = 0;
      for (int64_t p = rp[(size_t)r]; p < rp[(size_t)r + 1]; ++p) s += vl[(size_t)p];
      for (int64_t p = rp[(size_t)r]; p < rp[(size_t)r + 1]; ++p) a[(size_t)p] = vl[(size_t)p] / s;
    }
    std::vector<int64_t> rpc(rp), clc(cl);
    PetscCall(MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, N, nc, rpc.data(), clc.data(), a.data(), toCart));
  }
  if (toMesh) {  // transpose, scaled by the column sums (the cells' covered volumes)
    std::vector<int64_t> tp((size_t)nc + 1, 0), tc((size_t)nnz);
    std::vector<double> colsum((size_t)nc, 0.0);
    for (int64_t p = 0; p < nnz; ++p) {
      tp[(size_t)cl[(size_t)p] + 1] += 1;
      colsum[(size_t)cl[(size_t)p]] += vl[(size_t)p];
    }
    for (int64_t c = 0; c < nc; ++c) tp[(size_t)c + 1] += tp[(size_t)c];
    std::vector<int64_t> fill(tp.begin(), tp.end() - 1);
    std::vector<PetscScalar> ta((size_t)nnz);
    for (int64_t r = 0; r < N; ++r)  // rows ascend, so each transposed row's columns ascend
      for (int64_t p = rp[(size_t)r]; p < rp[(size_t)r + 1]; ++p) {
        const int64_t c = cl[(size_t)p];
        const int64_t q = fill[(size_t)c]++;
        tc[(size_t)q] = r;
        ta[(size_t)q] = vl[(size_t)p] / colsum[(size_t)c];
      }
    PetscCall(MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, nc, N, tp.data(), tc.data(), ta.data(), toMesh));
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

// the remap is the identity when every Cartesian cell is exactly mesh cell i (same ordering)
static bool remap_is_identity(const cfp_mesh_s* m, int64_t N) {
  if (m->ncells() != N || (int64_t)m->cm_col.size() != N) return false;
  for (int64_t r = 0; r < N; ++r) {
    if (m->cm_rowptr[(size_t)r + 1] - m->cm_rowptr[(size_t)r] != 1 || m->cm_col[(size_t)m->cm_rowptr[(size_t)r]] != r)
      return false;
    if (std::fabs(m->cm_val[(size_t)m->cm_rowptr[(size_t)r]] - m->vol[(size_t)r]) > 1e-12 * m->vol[(size_t)r]) return false;
  }
  return true;
}

extern "C" PetscErrorCode getFFTPrec3DContextMesh(PetscInt ndim, PetscScalar dt, PetscScalar a_x, PetscScalar a_y,
                                                  PetscScalar a_z, cfp_mesh_t m, FFTPrecTransportContext* ctx) {
  PetscFunctionBeginUser;
  PetscCheck(m && ctx, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "getFFTPrec3DContextMesh: NULL argument");
  PetscCheck(ndim == 3, PETSC_COMM_SELF, PETSC_ERR_SUP, "unstructured meshes are 3-D here (tetrahedra, hexahedra)");
  const double* b = m->bbox;
  PetscCall(getFFTPrec3DContext(ndim, dt, m->ncells(), a_x, a_y, a_z, b[0], b[2], b[4], b[1], b[3], b[5], ctx));
  Mat toCart = nullptr, toMesh = nullptr;
  PetscCall(MatCreateMeshCartesianRemap(m, ctx->n_x, ctx->n_y, ctx->n_z, b, nullptr, nullptr));
  if (!remap_is_identity(m, ctx->n_x * ctx->n_y * ctx->n_z)) {
    PetscCall(MatCreateMeshCartesianRemap(m, ctx->n_x, ctx->n_y, ctx->n_z, b, &toCart, &toMesh));
  }
  ctx->intersectionMatrix = toCart;
  PetscCall(FFTPrecTransportContextSetRemapBack(ctx, toMesh));
  PetscFunctionReturn(PETSC_SUCCESS);
}

extern "C" PetscErrorCode FFTPrec3DContextDestroyRemap(FFTPrecTransportContext* ctx) {
  PetscFunctionBeginUser;
  if (!ctx) PetscFunctionReturn(PETSC_SUCCESS);
  PetscCall(MatDestroy(&ctx->intersectionMatrix));
  Mat back = nullptr;
  PetscCall(FFTPrecTransportContextGetRemapBack(ctx, &back));
  PetscCall(MatDestroy(&back));
  PetscCall(FFTPrecTransportContextSetRemapBack(ctx, nullptr));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// initial_conditions_shock, src/TransportEquation.cxx:25-73 (the centre is the bounding box's)
extern "C" PetscErrorCode initial_conditions_shock_mesh(cfp_mesh_t m, Vec U) {
  PetscFunctionBeginUser;
  PetscCheck(m, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "NULL mesh");
  PetscInt n;
  PetscCall(VecGetLocalSize(U, &n));
  PetscCheck(n == m->ncells(), PETSC_COMM_SELF, PETSC_ERR_ARG_SIZ, "U size differs from the cell count");
  const double cx = (m->bbox[0] + m->bbox[1]) / 2, cy = (m->bbox[2] + m->bbox[3]) / 2, cz = (m->bbox[4] + m->bbox[5]) / 2;
  PetscScalar* u;
  PetscCall(VecGetArrayWrite(U, &u));
  for (int64_t j = 0; j < n; ++j) {
    const double* g = &m->ctr[(size_t)(3 * j)];
    const double r2 = (g[0] - cx) * (g[0] - cx) + (g[1] - cy) * (g[1] - cy) + (g[2] - cz) * (g[2] - cz);
    u[j] = std::sqrt(r2) < 0.3 ? 650.0 : 600.0;
  }
  PetscCall(VecRestoreArrayWrite(U, &u));
  PetscFunctionReturn(PETSC_SUCCESS);
}

// TransportEquation_impl_mpi with Mesh(filename): the same loop as TransportEquationGMRES
// (transport_cartesian.cpp) with the operator assembled over the mesh faces and the PCSHELL's
// context made from the mesh (remap to / from the Cartesian FFT grid).
extern "C" PetscErrorCode TransportEquationGMRESMesh(cfp_mesh_t m, const cfp_transport_config* cfg,
                                                     cfp_transport_result* res, double* U_out) {
  PetscFunctionBeginUser;
  PetscCheck(m && cfg && res, PETSC_COMM_SELF, PETSC_ERR_ARG_NULL, "TransportEquationGMRESMesh: NULL argument");
  PetscCheck(cfg->pc == CFP_TRANSPORT_PC_NONE || cfg->on_device, PETSC_COMM_SELF, PETSC_ERR_SUP,
             "the FFT preconditioner runs on HIP vectors only");
  std::memset((void*)res, 0, sizeof(*res));
  const double t_setup = wall();
  const PetscInt N = m->ncells();
  const double anorm = std::sqrt(cfg->a[0] * cfg->a[0] + cfg->a[1] * cfg->a[1] + cfg->a[2] * cfg->a[2]);
  PetscCheck(anorm > 0, PETSC_COMM_SELF, PETSC_ERR_ARG_OUTOFRANGE, "transport velocity is zero");
  double dx_min;
  {
    const int rc = cfp_mesh_min_ratio_vol_surf(m, &dx_min);
    PetscCheck(rc == CFP_SUCCESS, PETSC_COMM_SELF, rc, cfp_last_error());
  }
  const double dt = cfg->cfl * dx_min / anorm;  // :51-52
  res->dt = dt;

  Vec Un, dUn;
  if (cfg->on_device) PetscCall(VecCreateSeqHIP(PETSC_COMM_SELF, N, &Un));
  else PetscCall(VecCreateSeq(PETSC_COMM_SELF, N, &Un));
  PetscCall(VecDuplicate(Un, &dUn));
  PetscCall(initial_conditions_shock_mesh(m, Un));

  Mat A;
  {
    std::vector<int64_t> rp, cl;
    std::vector<double> vl;
    transport_rows(m, dt, cfg->a, cfg->sign_mode, 0.0, rp, cl, vl);
    PetscCall(MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, N, N, rp.data(), cl.data(),
                                        reinterpret_cast<PetscScalar*>(vl.data()), &A));
  }
  PetscCall(MatShift(A, 1.0));  // :117

  KSP ksp;
  PC pc;
  PetscCall(KSPCreate(PETSC_COMM_WORLD, &ksp));
  PetscCall(KSPSetType(ksp, KSPGMRES));
  PetscCall(KSPSetTolerances(ksp, cfg->precision, cfg->precision, PETSC_DEFAULT, cfg->max_its));
  PetscCall(KSPGMRESSetRestart(ksp, cfg->restart > 0 ? cfg->restart : 30));
  PetscCall(KSPSetPCSide(ksp, (PCSide)cfg->pc_side));
  PetscCall(KSPGetPC(ksp, &pc));
  FFTPrecTransportContext ctx;
  std::memset((void*)&ctx, 0, sizeof(ctx));
  if (cfg->pc == CFP_TRANSPORT_PC_FFT) {
    PetscCall(getFFTPrec3DContextMesh(3, dt, cfg->a[0], cfg->a[1], cfg->a[2], m, &ctx));
    if (cfg->lambda_mode == CFP_LAMBDA_MATCHED) {
      const double* b = m->bbox;
      ctx.lambda_x = cfg->a[0] * dt * (double)ctx.n_x / (b[1] - b[0]);
      ctx.lambda_y = cfg->a[1] * dt * (double)ctx.n_y / (b[3] - b[2]);
      ctx.lambda_z = cfg->a[2] * dt * (double)ctx.n_z / (b[5] - b[4]);
    }
    PetscCall(PCSetType(pc, PCSHELL));
    PetscCall(PCShellSetContext(pc, &ctx));
    PetscCall(PCShellSetSetUp(pc, setupFFTPrec3D));
    PetscCall(PCShellSetApply(pc, applyFFT3DPrecTransport));
    PetscCall(PCShellSetDestroy(pc, destroyFFTPrec3D));
    PetscCall(PCShellSetName(pc, "circulant FFT (HIP), mesh remap"));
    res->lambda[0] = ctx.lambda_x.real();
    res->lambda[1] = ctx.lambda_y.real();
    res->lambda[2] = ctx.lambda_z.real();
  } else {
    PetscCall(PCSetType(pc, PCNONE));
  }
  PetscCall(KSPSetOperators(ksp, A, A));
  PetscCall(KSPSetUp(ksp));
  PetscCall(KSPMiniSetUpWork(ksp, Un));
  PetscCall(MatMult(A, Un, dUn));
  if (cfg->on_device)
    PetscCheck(cfp_stream_sync(nullptr) == CFP_SUCCESS, PETSC_COMM_SELF, PETSC_ERR_LIB, "stream sync failed");
  res->setup_seconds = wall() - t_setup;

  int64_t it = 0;
  double time = 0.0;
  bool stationary = false;
  res->all_converged = 1;
  res->min_step_its = -1;
  while (it < cfg->ntmax && time <= cfg->tmax && !stationary) {  // :131
    PetscCall(VecCopy(Un, dUn));
    const double v = wall();
    PetscCall(KSPSolve(ksp, Un, Un));
    const double w = wall();
    PetscCall(VecAXPY(dUn, -1.0, Un));
    time += dt;
    it += 1;
    PetscReal norm;
    PetscCall(VecNorm(dUn, NORM_2, &norm));
    stationary = norm < cfg->precision;
    KSPConvergedReason reason;
    PetscInt its;
    PetscReal residu;
    PetscCall(KSPGetConvergedReason(ksp, &reason));
    PetscCall(KSPGetIterationNumber(ksp, &its));
    PetscCall(KSPGetResidualNorm(ksp, &residu));
    PetscInt calls;
    PetscLogDouble pcs;
    PetscCall(KSPMiniGetPCApplyStats(ksp, &calls, &pcs));
    res->solve_seconds += w - v;
    res->pc_seconds += pcs;
    res->pc_calls += calls;
    res->total_its += its;
    res->max_step_its = std::max<int64_t>(res->max_step_its, its);
    res->min_step_its = res->min_step_its < 0 ? its : std::min<int64_t>(res->min_step_its, its);
    res->last_reason = (int)reason;
    res->last_residual = residu;
    res->last_norm_dU = norm;
    if (reason != KSP_CONVERGED_RTOL && reason != KSP_CONVERGED_ATOL) res->all_converged = 0;
  }
  res->steps = it;
  res->time = time;
  if (U_out) {
    const PetscScalar* u;
    PetscCall(VecGetArrayRead(Un, &u));
    std::memcpy(U_out, (const void*)u, sizeof(double) * 2 * (size_t)N);
    PetscCall(VecRestoreArrayRead(Un, &u));
  }
  PetscCall(KSPDestroy(&ksp));
  PetscCall(FFTPrec3DContextDestroyRemap(&ctx));
  PetscCall(MatDestroy(&A));
  PetscCall(VecDestroy(&Un));
  PetscCall(VecDestroy(&dUn));
  PetscFunctionReturn(PETSC_SUCCESS);
}
#endif  // CFP_WITH_PETSC
