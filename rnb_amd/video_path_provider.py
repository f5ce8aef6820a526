"""Video path iterators (reference: video_path_provider.py:1-14)."""
import itertools
import os


class VideoPathIterator:
    """Interface: ``__iter__`` yields video paths, ideally forever."""

    def __iter__(self):
        raise NotImplementedError


class DirectoryVideoPathIterator(VideoPathIterator):
    """Walks ``root/label/video`` and cycles forever (model.py:86-113)."""

    def __init__(self, root):
        videos = []
        for label in sorted(os.listdir(root)):
            ldir = os.path.join(root, label)
            if not os.path.isdir(ldir):
                continue
            for video in sorted(os.listdir(ldir)):
                videos.append(os.path.join(ldir, video))
        if not videos:
            raise RuntimeError("No video available under %s." % root)
        self.videos = videos

    def __iter__(self):
        return itertools.cycle(self.videos)


class SyntheticVideoPathIterator(VideoPathIterator):
    """Endless ``synthetic://<id>?frames=<n>`` paths.

    There is no dataset on the target machines, so synthetic paths stand in for
    Kinetics-400 files: the frame count of each "video" is drawn from the
    Kinetics 10-s clip range (250-300 frames at 25-30 fps) with a fixed seed,
    and the synthetic loader decodes these paths deterministically.
    """

    def __init__(self, seed=0, min_frames=250, max_frames=300):
        self.seed = seed
        self.min_frames = min_frames
        self.max_frames = max_frames

    def __iter__(self):
        import random
        rng = random.Random(self.seed)
        for i in itertools.count():
            yield "synthetic://%d?frames=%d" % (
                i, rng.randint(self.min_frames, self.max_frames))


def parse_synthetic_path(path):
    """``synthetic://<id>?frames=<n>`` -> (id, n). Raises ValueError otherwise."""
    if not isinstance(path, str) or not path.startswith("synthetic://"):
        raise ValueError("not a synthetic path: %r" % (path,))
    body = path[len("synthetic://"):]
    vid, _, query = body.partition("?")
    frames = 300
    for kv in query.split("&"):
        if kv.startswith("frames="):
            frames = int(kv[len("frames="):])
    return int(vid), frames
