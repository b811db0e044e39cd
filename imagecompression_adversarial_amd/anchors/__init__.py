"""Mirror of the reference's ``anchors`` package (anchors/model.py, anchors/balle.py, anchors/utils.py)."""
