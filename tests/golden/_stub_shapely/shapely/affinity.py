"""Imported by couplers_coor.py, unused by couplers_coor_full_color."""
