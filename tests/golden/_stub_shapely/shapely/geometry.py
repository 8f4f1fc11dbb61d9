"""Polygon / MultiPolygon / LineString / GeometryCollection stand-ins (see package docstring)."""
import numpy as np


class _Ring:
    def __init__(self, pts):
        self._pts = list(pts)

    @property
    def coords(self):
        return self._pts + self._pts[:1] if self._pts else []

    @property
    def xy(self):
        c = self.coords
        return np.array([p[0] for p in c]), np.array([p[1] for p in c])


class Polygon:
    geom_type = "Polygon"

    def __init__(self, shell=None):
        pts = [] if shell is None else [(float(p[0]), float(p[1])) for p in np.asarray(shell, dtype=float)]
        if len(pts) > 1 and pts[0] == pts[-1]:
            pts = pts[:-1]
        self._pts = pts
        self.exterior = _Ring(pts)
        self.interiors = []

    @property
    def is_empty(self):
        return len(self._pts) < 3

    is_valid = True

    def intersection(self, other):
        """Sutherland-Hodgman clip of self by the convex polygon `other`."""
        out = list(self._pts)
        clip = other._pts
        # orientation of the clip polygon (signed area)
        area = sum(clip[i - 1][0] * clip[i][1] - clip[i][0] * clip[i - 1][1] for i in range(len(clip)))
        sgn = 1.0 if area > 0 else -1.0
        for i in range(len(clip)):
            a, b = clip[i - 1], clip[i]
            inp, out = out, []
            if not inp:
                break

            def side(p):
                return sgn * ((b[0] - a[0]) * (p[1] - a[1]) - (b[1] - a[1]) * (p[0] - a[0]))

            for j in range(len(inp)):
                p, q = inp[j - 1], inp[j]
                sp, sq = side(p), side(q)
                if sq >= 0:
                    if sp < 0:
                        t = sp / (sp - sq)
                        out.append((p[0] + t * (q[0] - p[0]), p[1] + t * (q[1] - p[1])))
                    out.append(q)
                elif sp >= 0:
                    t = sp / (sp - sq)
                    out.append((p[0] + t * (q[0] - p[0]), p[1] + t * (q[1] - p[1])))
        return Polygon(out) if len(out) >= 3 else Polygon()


class MultiPolygon:
    geom_type = "MultiPolygon"

    def __init__(self, polys=()):
        self.geoms = list(polys)

    @property
    def is_empty(self):
        return not self.geoms


class GeometryCollection(MultiPolygon):
    geom_type = "GeometryCollection"


class LineString:
    geom_type = "LineString"

    def __init__(self, coords):
        self._pts = [(float(p[0]), float(p[1])) for p in np.asarray(coords, dtype=float)]

    @property
    def xy(self):
        return np.array([p[0] for p in self._pts]), np.array([p[1] for p in self._pts])

    def simplify(self, tolerance, preserve_topology=True):
        pts = self._pts

        def dp(lo, hi, keep):
            ax, ay = pts[lo]
            bx, by = pts[hi]
            dx, dy = bx - ax, by - ay
            L = np.hypot(dx, dy)
            best, k = -1.0, -1
            for i in range(lo + 1, hi):
                px, py = pts[i]
                d = abs(dy * (px - ax) - dx * (py - ay)) / L if L > 0 else np.hypot(px - ax, py - ay)
                if d > best:
                    best, k = d, i
            if k >= 0 and best > tolerance:
                keep[k] = True
                dp(lo, k, keep)
                dp(k, hi, keep)

        keep = [False] * len(pts)
        if pts:
            keep[0] = keep[-1] = True
            dp(0, len(pts) - 1, keep)
        return LineString([p for p, k in zip(pts, keep) if k])
