from .layers import Conv2d, Linear, FlatSpace, flat_space
from .simple_cnn import SimpleCNN, reference_simple_cnn, param_count
from .resnet import ResNet, resnet18

__all__ = ["Conv2d", "Linear", "FlatSpace", "flat_space", "SimpleCNN", "reference_simple_cnn",
           "param_count", "ResNet", "resnet18"]
