"""pytest plugin (debug only): turn off switchml_amd.client._ready, to show
that tests/test_client_gpu.py::test_allreduce_waits_for_the_producing_stream
catches a client that does not make torch tensors ready before submitting."""


def pytest_collection_finish(session):
    import switchml_amd.client as c
    c._ready = lambda *a: None
