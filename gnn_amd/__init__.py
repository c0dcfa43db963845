"""gnn_amd — MI355X-native SpMM aggregation + feature placement path for mini-batch GNN
training (LADIES / GraphSAGE / GCN), a drop-in for HPC-Research-Lab/GNN's
``custom_sparse_ops`` operator and the training path around it. See DESIGN.md."""
__version__ = "0.1.0"
