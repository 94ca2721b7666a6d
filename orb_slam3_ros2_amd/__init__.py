"""orb_slam3_ros2_amd — MI355X-native ORB front-end + bundle-adjustment back-end.

Host-side mirror of the reference's hot-path interfaces over the C-ABI of
``liborbhip.so`` (include/orbhip.h):

  ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)      U:src/ORBextractor.cc
      __call__(image, mask, vLappingArea) -> (monoIndex, keypoints, descriptors)
  ORBmatcher.DescriptorDistance(a, b)                                       U:src/ORBmatcher.cc
  ORBmatcher(nnratio, checkOri).match_bf(...)                               (a12 rule)
  Optimizer.LocalBundleAdjustment(problem)                                  U:src/Optimizer.cc
  Optimizer.PoseOptimization(frame_problem)                                 U:src/Optimizer.cc
  ORBVocabulary(vocab).transform(desc)  (DBoW2 TemplatedVocabulary)         U:src/Frame.cc::ComputeBoW
  ORBmatcher.SearchByBoW(...)                                               U:src/ORBmatcher.cc
  ORBmatcher.SearchForInitialization(...)                                   U:src/ORBmatcher.cc
  ORBmatcher.SearchByProjectionLastFrame / SearchLocalPoints(...)           U:src/ORBmatcher.cc
  KeyFrameDatabase(max_kf).DetectRelocalizationCandidates / DetectNBestCandidates
                                                                            U:src/KeyFrameDatabase.cc
  FrameStream(w, h, frames_in_flight).push(frame)   Frame ctor -> ExtractORB + match to the last
                                                    frame, pipelined on the device

The HIP library is the only compute path: importing this package on a box without the
built extension, or calling it without a GPU, raises — there is no CPU fallback.
"""
from __future__ import annotations

from ._lib import OrbHipError, lib, library_path  # noqa: F401
from .extractor import KeyPoint, ORBextractor  # noqa: F401
from .matcher import ORBmatcher  # noqa: F401
from .optimizer import BAProblem, BAResult, Optimizer, PoseProblem, PoseResult  # noqa: F401
from .bow import ORBVocabulary  # noqa: F401
from .kfdb import KeyFrameDatabase  # noqa: F401
from .frontend import FrameStream  # noqa: F401
from .camera import PinholeCamera  # noqa: F401

__all__ = ["ORBextractor", "KeyPoint", "ORBmatcher", "Optimizer", "BAProblem", "BAResult", "PoseProblem", "PoseResult", "ORBVocabulary", "KeyFrameDatabase", "FrameStream", "PinholeCamera",
           "OrbHipError",
           "lib", "library_path"]
