"""Models package — MI355X-native drop-in for reference src/models/__init__.py (hot-path subset:
GNN, ShellConvolutionLayer and the pooling layers)."""
from .gnn import GNN, GNNConfig
from .layers import LinearBlock, MultiLayerPerceptron, ShellConvolutionLayer
from .losses import L1Loss, WeightedL1Loss
from .pooling import (MaxPoolingLayer, MeanPoolingLayer, MultiHeadAttentionPoolingLayer, SetAttentionPoolingLayer,
                      SumPoolingLayer, create_pooling_layer)

__all__ = [
    "GNN", "GNNConfig", "ShellConvolutionLayer", "LinearBlock", "MultiLayerPerceptron",
    "MeanPoolingLayer", "MaxPoolingLayer", "SumPoolingLayer", "MultiHeadAttentionPoolingLayer",
    "SetAttentionPoolingLayer", "create_pooling_layer", "L1Loss", "WeightedL1Loss",
]
