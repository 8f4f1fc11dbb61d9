"""Throwaway planar stand-in for the few shapely calls couplers_coor.py makes (test-only).

Used by tests/golden/gen_golden.py to run the reference geometry function unmodified so that
its shapely-free tables (lut_gap, lut_TIR, lut_Fresnel, eff_reg_FOV*, IC, the angles and
k-vectors) can be pinned.  Clipping is Sutherland-Hodgman against the (convex) band and
simplify is Douglas-Peucker: the FC / OC / eff_reg* polygons it yields follow these
semantics, not GEOS's, and are not claimed as reference outputs.
"""
