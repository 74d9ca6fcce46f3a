"""graphneuralnetwork_amd -- MI355X-native message-passing aggregation for the
GCN / GAT / GraphSAGE forward paths of kaddly/GraphNeuralNetwork.

Drop-in modules (same class names, constructor args, forward signatures and
state_dict keys as the reference):

* ``graphneuralnetwork_amd.gcn``       -- GCN_Model, Graph_conv_layer      (GCN/GCN.py)
* ``graphneuralnetwork_amd.gat``       -- GraphAttentionLayer, SpGraphAttentionLayer,
                                          GAT, SpGAT                       (GAT/models/*.py)
* ``graphneuralnetwork_amd.graphsage`` -- SageLayer, GraphSAGE, Aggregator (GraphSAGE/*.py)

The aggregation hot paths run as hand-written gfx950 HIP kernels in
``lib/libgnn_mi355x.so`` behind the C-ABI of ``include/gnn_mi355x.h``.
"""
__version__ = "0.1.0"
