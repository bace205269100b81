"""FE matrix source: meshes, P1 + Morley varfs and the 26-matrix block layout."""
from .mesh import TriMesh, strip_mesh, disc_nodes, locate_points
from .varf import plate_varfs, MorleyBasis
from .layout import load_matrices_unsymm, block_layout
