"""MLPs: Criteo ``confA`` and the reference's ``sanity`` net.

``confA`` (reference ``cerebro_gpdb/in_rdbms_helper.py:419-424``,
``cerebro_gpdb/run_pytorchddp.py:300-307``): Dense 7306->1000 ReLU ->
1000->500 ReLU -> 500->2 softmax; 7 808 502 parameters.  Its input is a
0/1 one-hot of 13 bucketised + 26 hashed features (exactly 39 ones per row,
SURVEY.md A14), so layer 1 is an *embedding-bag sum* of 39 weight rows
(``ops.nn.embedding_bag``) — identical math to the dense GEMM on the one-hot
input at 1/187th of the FLOPs and bytes.

``sanity`` (``in_rdbms_helper.py:414-418``): Dense 4->10 ReLU -> 10->10 ReLU
-> 10->3 softmax on dense 4-feature input.
"""

from .common import Dense, PackedNet
from ..config.catalog import INPUT_SHAPE_CRITEO, NUM_CLASSES_CRITEO
from ..ops import nn as P
from ..runtime.arena import ParamSpec


class PackedConfA(PackedNet):
    input_kind = "sparse"

    def __init__(self, in_dim=INPUT_SHAPE_CRITEO[0], num_classes=NUM_CLASSES_CRITEO):
        super(PackedConfA, self).__init__()
        self.in_dim = in_dim
        self.num_classes = num_classes
        # Keras Dense kernel layout [in, out]: one contiguous row per input column
        self.w1 = self.spec(ParamSpec("dense_1/kernel", (in_dim, 1000), "weight", init="glorot",
                                      fan_in=in_dim, fmt="keras"))
        self.b1 = self.spec(ParamSpec("dense_1/bias", (1000,), "bias"))
        self.fc2 = Dense(self, "dense_2", 1000, 500)
        self.fc3 = Dense(self, "dense_3", 500, num_classes)
        self.build_layout()

    def forward(self, idx, training):
        x = P.embedding_bag(idx, self.ref(self.w1), self.ref(self.b1), relu=True, anchor=self.anchor)
        x = self.bucket_mark(x, self.fc2.w)
        x = self.dense(x, self.fc2, relu=True)
        x = self.bucket_mark(x, self.fc3.w)
        return self.dense(x, self.fc3)


class PackedSanity(PackedNet):
    input_kind = "dense"

    def __init__(self, in_dim=4, num_classes=3):
        super(PackedSanity, self).__init__()
        self.in_dim = in_dim
        self.num_classes = num_classes
        self.fc1 = Dense(self, "dense_1", in_dim, 10)
        self.fc2 = Dense(self, "dense_2", 10, 10)
        self.fc3 = Dense(self, "dense_3", 10, num_classes)
        self.build_layout()

    def forward(self, x, training):
        x = self.dense(x, self.fc1, relu=True, anchor=True)
        x = self.bucket_mark(x, self.fc2.w)
        x = self.dense(x, self.fc2, relu=True)
        x = self.bucket_mark(x, self.fc3.w)
        return self.dense(x, self.fc3)
