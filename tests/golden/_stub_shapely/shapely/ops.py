def unary_union(geoms):
    raise NotImplementedError("not used by couplers_coor_full_color")


def polygonize(lines):
    raise NotImplementedError("not used by couplers_coor_full_color")
