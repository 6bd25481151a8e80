"""The four workloads ("model families") of the suite, each with a single-device
form and a row/shard-decomposed multi-GPU form:

  lab1  VectorSub / ShardedVectorSub           element-wise fp64/fp32 c = a - b
  lab2  EdgeDetector / SlabEdgeDetector        Roberts cross + KxK convolutions
  lab3  PixelClassifier / SlabPixelClassifier  Mahalanobis ML classification
  stencil  SlabJacobi                          2-D Jacobi with halo exchange
"""

from .classifier import PixelClassifier, SlabPixelClassifier
from .edge import EdgeDetector, SlabEdgeDetector
from .jacobi import SlabJacobi
from .vector import ShardedVectorSub, VectorSub

__all__ = ["PixelClassifier", "SlabPixelClassifier", "EdgeDetector", "SlabEdgeDetector", "SlabJacobi",
           "ShardedVectorSub", "VectorSub"]
