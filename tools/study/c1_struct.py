"""VERDICT r03 item 2's scene-structure specialisation, measured on the Cornell kernel: when the scene is the README
Cornell box's structure (rows Cube, Cornellbox, Sphere), the primary/secondary sweep is straight-line code over the
three rows with their types as constants (no per-row type dispatch, no loop), as a kernel compiled for the scene's
primitive sequence would run it. Same operations in the same order: bit-identical."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [("""  for (int i = 0; i < c.n; i++) {
    V3 hl = v3s(0.0f);
    const float t = primT(c, PRIM(c, i), r, &hl);
    if (t < best) { best = t; bi = i; bhl = hl; }
  }
  Sweep sw; sw.best = best; sw.bi = bi; sw.bhl = bhl;
  return sw;
}""", """  if (c.kShapes == SAIL_KSET_CORNELL_SHAPES && c.n == 3 && PRIM(c, 0).type == SAIL_CUBE &&
      PRIM(c, 1).type == SAIL_CORNELLBOX && PRIM(c, 2).type == SAIL_SPHERE) {
    { const float t = cubeT(PRIM(c, 0), r); if (t < best) { best = t; bi = 0; bhl = v3s(0.0f); } }
    { const float t = cornellT(PRIM(c, 1), r); if (t < best) { best = t; bi = 1; bhl = v3s(0.0f); } }
    { V3 hl = v3s(0.0f); const float t = sphereT(PRIM(c, 2), r, &hl); if (t < best) { best = t; bi = 2; bhl = hl; } }
  } else
  for (int i = 0; i < c.n; i++) {
    V3 hl = v3s(0.0f);
    const float t = primT(c, PRIM(c, i), r, &hl);
    if (t < best) { best = t; bi = i; bhl = hl; }
  }
  Sweep sw; sw.best = best; sw.bi = bi; sw.bhl = bhl;
  return sw;
}""")])
