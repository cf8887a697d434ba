from simclr_pytorch_distributed_amd.utils.tb import Logger, crc32c, read_events


def test_crc32c_known_vector():
    assert crc32c(b"123456789") == 0xE3069283


def test_event_roundtrip(tmp_path):
    lg = Logger(str(tmp_path), flush_secs=0)
    lg.log_value("loss", 1.5, 3)
    lg.log_value("info/norm_mean", 2.25, 4)
    lg.close()
    ev = read_events(lg.path)
    assert (3, "loss", 1.5) in ev and (4, "info/norm_mean", 2.25) in ev
