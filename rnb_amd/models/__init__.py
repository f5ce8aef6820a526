"""Model families. ``r2p1d``: R(2+1)D-10/18/26/34 video classification."""
