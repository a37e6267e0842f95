"""Viewer stand-in (rendering is out of scope)."""
PlantOS3DViewer = None
