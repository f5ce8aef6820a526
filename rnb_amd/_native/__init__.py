"""Built native libraries live here (librnb_*.so, git-ignored, built in-tree
by ``python -m rnb_amd.build`` / ``__graft_entry__.build()``)."""
