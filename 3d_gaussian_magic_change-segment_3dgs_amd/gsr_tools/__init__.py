"""Harness helpers for the gsr rasterizer: reference camera conventions and the
synthetic scenes of SURVEY.md s8(d).  Not part of the drop-in API."""
