"""Model-selection-tuple (MST) identifiers.

* ``mst_2_str`` — the CTQ checkpoint file key
  (reference ``cerebro_gpdb/in_rdbms_helper.py:232-235``)
* ``mst2key`` / ``key2mst`` — the sorted ``k:v|k:v`` key
  (reference ``cerebro_gpdb/utils.py:58-86``)
"""


def mst_2_str(mst):
    s = "learning_rate:{},lambda_value:{},batch_size:{},model:{}".format(
        mst["learning_rate"], mst["lambda_value"], mst["batch_size"], mst["model"])
    if mst.get("optimizer", "adam") != "adam":     # extension: keeps Adam keys reference-exact
        s += ",optimizer:{}".format(mst["optimizer"])
    return s


def mst2key(mst):
    parts = []
    for k in sorted(mst.keys()):
        parts.append("{}:{}".format(k, mst[k]))
    return "|".join(parts).replace(" ", "_")


def key2mst(key):
    mst = {}
    for item in key.split("|"):
        name, value = item.split(":", 1)
        if name == "batch_size":
            value = int(value)
        elif name == "model":
            pass
        else:
            value = float(value)
        mst[name] = value
    return mst


def model_key(index, mst):
    """CTQ model key: ``{i}_{mst_2_str(mst)}`` (reference ctq.py:326-333)."""
    return "{}_{}".format(index, mst_2_str(mst))
