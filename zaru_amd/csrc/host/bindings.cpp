// bindings.cpp -- pybind11 module `_zaru_host`: the reference's host-side API (Detector,
// NonMaxSuppression, Estimator, LandmarkTracker, Rect/RotatedRect, ...) over the C ABI, so
// that parity tests read like the reference's own #[test]s.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "detection.h"
#include "hand_tracker.h"
#include "device_hand_tracker.h"
#include "landmark.h"
#include "pipeline.h"
#include "device_face_loop.h"
#include "device_tracker.h"

namespace py = pybind11;
using namespace zh;

namespace {

Image host_image(const py::array_t<uint8_t, py::array::c_style> &a) {
    if (a.ndim() != 3 || a.shape(2) != 4) throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "image must be HxWx4 uint8 RGBA");
    Image im;
    im.rgba = a.data();
    im.height = (uint32_t)a.shape(0);
    im.width = (uint32_t)a.shape(1);
    im.row_stride = (uint64_t)a.shape(1) * 4;
    im.on_device = false;
    return im;
}

py::tuple rect_tuple(const Rect &r) {
    return py::make_tuple(r.center().x, r.center().y, r.width(), r.height());
}

py::dict estimate_dict(const Estimate &e) {
    py::dict d;
    py::array_t<float> p({(py::ssize_t)e.size(), (py::ssize_t)3});
    std::memcpy(p.mutable_data(), e.positions.data(), e.positions.size() * 4);
    d["landmarks"] = p;
    d["confidence"] = e.confidence;
    d["raw_handedness"] = e.raw_handedness;
    d["tongue_out"] = e.tongue_out;
    py::array_t<float> w({(py::ssize_t)(e.world.size() / 3), (py::ssize_t)3});
    if (!e.world.empty()) std::memcpy(w.mutable_data(), e.world.data(), e.world.size() * 4);
    d["world"] = w;  // hand metric landmarks (Identity_3); empty for the other networks
    return d;
}

DetectorNetwork detector_net(const std::string &name) {
    if (name == "face") return DetectorNetwork::short_range_face();
    if (name == "face_full") return DetectorNetwork::full_range_face();
    if (name == "palm") return DetectorNetwork::palm_lite();
    throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "detector network must be 'face', 'face_full' or 'palm'");
}

LandmarkNetwork landmark_net(const std::string &name) {
    if (name == "facemesh") return LandmarkNetwork::face_mesh_v1();
    if (name == "facemesh_v2") return LandmarkNetwork::face_mesh_v2();
    if (name == "hand") return LandmarkNetwork::hand_lite();
    if (name == "eye") return LandmarkNetwork::eye();
    if (name == "face68_pfld") return LandmarkNetwork::face_onnx_68();
    if (name == "face68_peppa") return LandmarkNetwork::peppa_68();
    throw ZaruError(ZR_ERR_INVALID_ARGUMENT,
                    "landmark network must be 'facemesh', 'facemesh_v2', 'hand', 'eye', 'face68_pfld' or 'face68_peppa'");
}

// Detector::detect_impl after inference on raw outputs (detection.rs:231-267)
std::vector<Detection> detect_post(const std::string &net, py::array_t<float, py::array::c_style> boxes,
                                   py::array_t<float, py::array::c_style> logits, uint32_t img_w,
                                   uint32_t img_h, float thresh, float iou, bool remove) {
    DetectorNetwork dn = detector_net(net);
    // network input sizes: short range 128, full range / palm 192 (the ONNX input shapes)
    const uint32_t s = dn.kind == NetworkKind::FaceDetectionShortRange ? 128 : 192;
    if ((size_t)logits.size() != dn.anchors().size() || (size_t)boxes.size() != dn.anchors().size() * dn.params)
        throw ZaruError(ZR_ERR_SHAPE, "raw outputs do not match the network's anchors");
    std::vector<Detection> raw;
    dn.extract(boxes.data(), logits.data(), thresh, s, s, raw);
    NonMaxSuppression nms;
    nms.set_iou_thresh(iou);
    if (remove) nms.set_mode(SuppressionMode::Remove);
    auto out = nms.process(raw);
    Rect rect;
    letterbox_view(img_w, img_h, AspectRatio::of(s, s), &rect);
    map_detections(out, rect, s);
    return out;
}

}  // namespace

PYBIND11_MODULE(_zaru_host, m) {
    m.doc() = "Host-side mirror of Zaru's detection/landmark API over the MI355X C ABI";
    py::register_exception<ZaruError>(m, "ZaruError", PyExc_RuntimeError);

    py::class_<Rect>(m, "Rect")
        .def_static("from_center", &Rect::from_center)
        .def_static("from_top_left", &Rect::from_top_left)
        .def_static("bounding", [](const std::vector<std::pair<float, float>> &pts) -> py::object {
            std::vector<Vec2> v;
            for (auto &p : pts) v.push_back({p.first, p.second});
            Rect r;
            if (!Rect::bounding(v.data(), v.size(), r)) return py::none();
            return py::cast(r);
        })
        .def_property_readonly("center", [](const Rect &r) { return py::make_tuple(r.center().x, r.center().y); })
        .def_property_readonly("size", [](const Rect &r) { return py::make_tuple(r.width(), r.height()); })
        .def("width", &Rect::width)
        .def("height", &Rect::height)
        .def("x", &Rect::x)
        .def("y", &Rect::y)
        .def("area", &Rect::area)
        .def("top_left", [](const Rect &r) { return py::make_tuple(r.top_left().x, r.top_left().y); })
        .def("scale", &Rect::scale)
        .def("grow_rel", &Rect::grow_rel)
        .def("grow_to_fit_aspect", [](const Rect &r, uint32_t w, uint32_t h) { return r.grow_to_fit_aspect(AspectRatio::of(w, h)); })
        .def("iou", &Rect::iou)
        .def("intersection", [](const Rect &a, const Rect &b) -> py::object {
            Rect o;
            if (!a.intersection(b, o)) return py::none();
            return py::cast(o);
        })
        .def("intersection_area", &Rect::intersection_area)
        .def("contains_point", [](const Rect &r, float x, float y) { return r.contains_point({x, y}); })
        .def("tuple", &rect_tuple)
        .def("__eq__", &Rect::operator==)
        .def("__repr__", [](const Rect &r) {
            return "Rect @ (" + std::to_string(r.center().x) + "," + std::to_string(r.center().y) + ")/" +
                   std::to_string(r.width()) + "x" + std::to_string(r.height());
        });

    py::class_<RotatedRect>(m, "RotatedRect")
        .def(py::init<Rect, float>(), py::arg("rect"), py::arg("radians") = 0.f)
        .def_static("bounding", [](float rad, const std::vector<std::pair<float, float>> &pts) -> py::object {
            std::vector<Vec2> v;
            for (auto &p : pts) v.push_back({p.first, p.second});
            RotatedRect r;
            if (!RotatedRect::bounding(rad, v.data(), v.size(), 2, r)) return py::none();
            return py::cast(r);
        })
        .def("rect", &RotatedRect::rect)
        .def("rotation_radians", &RotatedRect::rotation_radians)
        .def("grow_rel", &RotatedRect::grow_rel)
        .def("transform_in", [](const RotatedRect &r, float x, float y) { auto p = r.transform_in({x, y}); return py::make_tuple(p.x, p.y); })
        .def("transform_out", [](const RotatedRect &r, float x, float y) { auto p = r.transform_out({x, y}); return py::make_tuple(p.x, p.y); })
        .def("contains_point", [](const RotatedRect &r, float x, float y) { return r.contains_point({x, y}); });

    py::class_<ViewData>(m, "ViewData")
        .def_static("full", &ViewData::full)
        .def("view", [](const ViewData &v, const RotatedRect &r) { return v.view(r); })
        .def("view_rect", [](const ViewData &v, const Rect &r) { return v.view(RotatedRect(r, 0.f)); })
        .def_property_readonly("rect", [](const ViewData &v) { return v.rect; })
        .def("local_rect", &ViewData::local_rect)
        .def("zr_view", [](const ViewData &v) {
            auto z = to_zr_view(v);
            return py::make_tuple(z.cx, z.cy, z.w, z.h, z.rad);
        });

    m.def("signed_angle_to", [](float ax, float ay, float bx, float by) { return signed_angle_to({ax, ay}, {bx, by}); });
    m.def("sigmoid", &sigmoid);
    m.def("letterbox_view", [](uint32_t w, uint32_t h, uint32_t aw, uint32_t ah) {
        Rect r;
        ViewData v = letterbox_view(w, h, AspectRatio::of(aw, ah), &r);
        return py::make_tuple(v, r);
    });
    m.def("candidate_logit_floor", &candidate_logit_floor);

    py::class_<Detection>(m, "Detection")
        .def(py::init([](float conf, const Rect &r, float angle,
                         const std::vector<std::pair<float, float>> &kps) {
                 Detection d;
                 d.confidence = conf;
                 d.rect = r;
                 d.angle = angle;
                 for (auto &k : kps) d.keypoints.push_back({k.first, k.second});
                 return d;
             }), py::arg("confidence"), py::arg("rect"), py::arg("angle") = 0.f,
             py::arg("keypoints") = std::vector<std::pair<float, float>>{})
        .def("confidence", [](const Detection &d) { return d.confidence; })
        .def("angle", [](const Detection &d) { return d.angle; })
        .def("bounding_rect", [](const Detection &d) { return d.rect; })
        .def_readonly("anchor", &Detection::anchor)
        .def("keypoints", [](const Detection &d) {
            std::vector<std::pair<float, float>> k;
            for (auto &p : d.keypoints) k.push_back({p.x, p.y});
            return k;
        });

    py::enum_<SuppressionMode>(m, "SuppressionMode")
        .value("Remove", SuppressionMode::Remove)
        .value("Average", SuppressionMode::Average);

    py::class_<NonMaxSuppression>(m, "NonMaxSuppression")
        .def(py::init<>())
        .def("set_iou_thresh", &NonMaxSuppression::set_iou_thresh)
        .def("set_mode", &NonMaxSuppression::set_mode)
        .def("process", [](const NonMaxSuppression &n, std::vector<Detection> dets) { return n.process(dets); });

    m.def("detect_post", &detect_post, py::arg("network"), py::arg("boxes"), py::arg("logits"),
          py::arg("img_w"), py::arg("img_h"), py::arg("thresh") = Detector::DEFAULT_THRESHOLD,
          py::arg("iou") = NonMaxSuppression::DEFAULT_IOU_THRESH, py::arg("remove") = false);
    m.def("nms_ties", [](const std::string &net, py::array_t<float, py::array::c_style> logits, float thresh) {
        // NonMaxSuppression::TieCount of a frame's candidates: (candidates, tied)
        DetectorNetwork dn = detector_net(net);
        if ((size_t)logits.size() != dn.anchors().size()) throw ZaruError(ZR_ERR_SHAPE, "one logit per anchor");
        std::vector<Detection> raw;
        for (size_t i = 0; i < dn.anchors().size(); i++) {
            const float c = sigmoid(logits.data()[i]);
            if (c < thresh) continue;
            Detection d;
            d.confidence = c;
            raw.push_back(d);
        }
        NonMaxSuppression::TieCount t;
        NonMaxSuppression().process(raw, &t);
        return std::make_pair(t.candidates, t.tied);
    }, py::arg("network"), py::arg("logits"), py::arg("thresh") = Detector::DEFAULT_THRESHOLD);
    m.def("anchors", [](const std::string &net) {
        auto a = detector_net(net).anchors();
        py::array_t<float> o({(py::ssize_t)a.size(), (py::ssize_t)2});
        std::memcpy(o.mutable_data(), a.data(), a.size() * 8);
        return o;
    });
    m.def("set_models_dir", &set_models_dir);
    m.def("pack_detection_records", [](const std::vector<std::vector<Detection>> &dets,
                                       const std::vector<uint32_t> &frame_ids, uint32_t rmax) {
        py::array_t<float> a({(py::ssize_t)dets.size(), (py::ssize_t)det_record_width(rmax)});
        pack_detection_records(dets, frame_ids, rmax, a.mutable_data());
        return a;
    }, py::arg("detections"), py::arg("frame_ids"), py::arg("rmax") = 8);

    py::class_<Detector>(m, "Detector")
        .def(py::init([](const std::string &net, int device) { return new Detector(detector_net(net), device); }),
             py::arg("network") = "face", py::arg("device") = 0)
        .def("set_threshold", &Detector::set_threshold)
        .def("set_nms_iou", [](Detector &d, float t) { d.nms_mut().set_iou_thresh(t); })
        .def("set_nms_mode", [](Detector &d, SuppressionMode m) { d.nms_mut().set_mode(m); })
        .def("input_width", &Detector::input_width)
        .def("detect", [](Detector &d, py::array_t<uint8_t, py::array::c_style> img) {
            return d.detect(host_image(img));
        });

    py::class_<Estimator>(m, "Estimator")
        .def(py::init([](const std::string &net, int device) { return new Estimator(landmark_net(net), device); }),
             py::arg("network") = "facemesh", py::arg("device") = 0)
        .def("input_width", &Estimator::input_width)
        .def("estimate", [](Estimator &e, py::array_t<uint8_t, py::array::c_style> img, const ViewData &v) {
            Image im = host_image(img);
            return estimate_dict(e.estimate(im, v));
        })
        .def("estimate_image", [](Estimator &e, py::array_t<uint8_t, py::array::c_style> img) {
            Image im = host_image(img);
            return estimate_dict(e.estimate(im, ViewData::full(im.width, im.height)));
        })
        .def("angle_radians", [](const Estimator &e, py::array_t<float, py::array::c_style> lm) {
            Estimate est;
            est.positions.assign(lm.data(), lm.data() + lm.size());
            return estimate_angle(e.network(), est);
        });

    py::class_<LandmarkTracker>(m, "LandmarkTracker")
        .def(py::init([](const std::string &net, int device) {
                 return new LandmarkTracker(Estimator(landmark_net(net), device));
             }), py::arg("network") = "facemesh", py::arg("device") = 0)
        .def("set_roi", [](LandmarkTracker &t, const RotatedRect &r) { t.set_roi(r); })
        .def("set_roi_rect", [](LandmarkTracker &t, const Rect &r) { t.set_roi(RotatedRect(r, 0.f)); })
        .def("set_loss_threshold", &LandmarkTracker::set_loss_threshold)
        .def("set_roi_padding", &LandmarkTracker::set_roi_padding)
        .def("roi", [](const LandmarkTracker &t) -> py::object {
            if (!t.roi()) return py::none();
            return py::cast(*t.roi());
        })
        .def("track", [](LandmarkTracker &t, py::array_t<uint8_t, py::array::c_style> img) -> py::object {
            auto r = t.track(host_image(img));
            if (!r) return py::none();
            py::dict d = estimate_dict(r->estimate);
            d["view_rect"] = r->view_rect;
            d["updated_roi"] = r->updated_roi;
            return d;
        });

    py::class_<HandTracker>(m, "HandTracker")
        .def(py::init<int>(), py::arg("device") = 0)
        .def("set_redetect_interval", &HandTracker::set_redetect_interval, py::arg("ms"))
        .def("set_iou_thresh", &HandTracker::set_iou_thresh)
        .def("set_loss_threshold", &HandTracker::set_loss_threshold)
        .def("track", [](HandTracker &t, py::array_t<uint8_t, py::array::c_style> img, py::object now_ms) {
                 Image im = host_image(img);
                 if (now_ms.is_none()) t.track(im);
                 else t.track(im, now_ms.cast<double>());
             }, py::arg("image"), py::arg("now_ms") = py::none())
        .def("hands", [](const HandTracker &t) {
            py::list out;
            for (const auto &h : t.hands()) {
                py::dict d = estimate_dict(h.landmarks);
                d["id"] = h.id;
                d["view_rect"] = h.view_rect;
                out.append(d);
            }
            return out;
        })
        .def("wait_detection", &HandTracker::wait_detection)
        .def("inject_detections", &HandTracker::inject_detections)
        .def("detection_running", &HandTracker::detection_running)
        .def("num_tracked", &HandTracker::num_tracked)
        .def_static("filter_detections", &HandTracker::filter_detections)
        .def_static("dedupe_rois", &HandTracker::dedupe_rois);

    // LandmarkTracker state on the device over n video streams
    py::class_<DeviceHandTracker>(m, "DeviceHandTracker")
        .def(py::init<size_t, int, int>(), py::arg("streams"), py::arg("slots") = 4, py::arg("device") = 0)
        .def("set_redetect_interval", &DeviceHandTracker::set_redetect_interval, py::arg("ms"))
        .def("set_iou_thresh", &DeviceHandTracker::set_iou_thresh)
        .def("set_loss_threshold", &DeviceHandTracker::set_loss_threshold)
        .def("set_palm_every_frame", &DeviceHandTracker::set_palm_every_frame, py::arg("on"))
        .def("palm_frames", &DeviceHandTracker::palm_frames)
        .def("inject_detections", &DeviceHandTracker::inject_detections)
        .def("step", [](DeviceHandTracker &t, const std::vector<std::tuple<uint64_t, uint32_t, uint32_t, uint64_t>> &frames,
                        double now_ms) {
            std::vector<Image> im;
            for (auto &f : frames) {
                Image i;
                i.rgba = reinterpret_cast<const uint8_t *>(std::get<0>(f));
                i.width = std::get<1>(f);
                i.height = std::get<2>(f);
                i.row_stride = std::get<3>(f);
                i.on_device = true;
                im.push_back(i);
            }
            py::gil_scoped_release nogil;
            t.step(im, now_ms);
        }, py::arg("frames"), py::arg("now_ms"))
        .def("synchronize", &DeviceHandTracker::synchronize, py::call_guard<py::gil_scoped_release>())
        .def("hand_counts", &DeviceHandTracker::hand_counts)
        .def("detection_pending", &DeviceHandTracker::detection_pending)
        .def("dropped_hands", &DeviceHandTracker::dropped_hands)
        .def("dropped_detections", &DeviceHandTracker::dropped_detections)
        .def("detection_capacity", &DeviceHandTracker::detection_capacity)
        .def("hands", [](DeviceHandTracker &t, size_t s) {
            py::list out;
            for (auto &h : t.hands(s)) {
                py::dict d;
                d["id"] = h.id;
                py::array_t<float> a({(py::ssize_t)(h.landmarks.size() / 3), (py::ssize_t)3});
                std::memcpy(a.mutable_data(), h.landmarks.data(), h.landmarks.size() * 4);
                d["landmarks"] = a;
                d["view_rect"] = h.view_rect;
                out.append(d);
            }
            return out;
        });
    py::class_<DeviceTracker>(m, "DeviceTracker")
        .def(py::init([](const std::string &net, int device, float padding, float loss) {
                 return new DeviceTracker(landmark_net(net), device, padding, loss);
             }), py::arg("network") = "facemesh", py::arg("device") = 0,
             py::arg("padding") = LandmarkTracker::DEFAULT_ROI_PADDING,
             py::arg("loss_threshold") = LandmarkTracker::DEFAULT_LOSS_THRESHOLD)
        .def("set_rois", [](DeviceTracker &t, const std::vector<std::tuple<float, float, float, float, float>> &rois,
                            const std::vector<std::pair<uint32_t, uint32_t>> &sizes) {
            std::vector<RotatedRect> r;
            for (auto &v : rois)
                r.emplace_back(Rect::from_center(std::get<0>(v), std::get<1>(v), std::get<2>(v), std::get<3>(v)),
                               std::get<4>(v));
            t.set_rois(r, sizes);
        })
        .def("step", [](DeviceTracker &t, const std::vector<std::tuple<uint64_t, uint32_t, uint32_t, uint64_t>> &frames) {
            std::vector<Image> im;
            for (auto &f : frames) {
                Image i;
                i.rgba = reinterpret_cast<const uint8_t *>(std::get<0>(f));
                i.width = std::get<1>(f);
                i.height = std::get<2>(f);
                i.row_stride = std::get<3>(f);
                i.on_device = true;
                im.push_back(i);
            }
            py::gil_scoped_release nogil;
            t.step(im);
        })
        .def("synchronize", &DeviceTracker::synchronize, py::call_guard<py::gil_scoped_release>())
        .def("__len__", &DeviceTracker::size)
        .def("states", [](DeviceTracker &t) {
            py::list out;
            for (const auto &s : t.states()) {
                py::dict d;
                d["roi"] = RotatedRect(Rect::from_center(s.roi[0], s.roi[1], s.roi[2], s.roi[3]), s.roi[4]);
                d["updated_roi"] = RotatedRect(Rect::from_center(s.updated[0], s.updated[1], s.updated[2], s.updated[3]), s.updated[4]);
                d["view_rect"] = RotatedRect(Rect::from_center(s.view_rect[0], s.view_rect[1], s.view_rect[2], s.view_rect[3]), s.view_rect[4]);
                d["active"] = s.active != 0;
                d["tracked"] = s.tracked != 0;
                d["confidence"] = s.confidence;
                out.append(d);
            }
            return out;
        })
        .def("views", [](DeviceTracker &t) {
            auto v = t.views();
            py::array_t<float> a({(py::ssize_t)v.size(), (py::ssize_t)10});
            static_assert(sizeof(zr_view_desc) == 40, "zr_view_desc");
            std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(zr_view_desc));
            return a;  // f32 view of {half_w, half_h, tl_x, tl_y, view_w, view_h, cos, sin, frame, pad}
        })
        .def("host_view", [](const DeviceTracker &t, const RotatedRect &roi, uint32_t fw, uint32_t fh, uint32_t frame) {
            const zr_view_desc d = t.host_view(roi, fw, fh, frame);
            py::array_t<float> a(10);
            std::memcpy(a.mutable_data(), &d, sizeof(d));
            return a;
        })
        .def("landmarks", [](DeviceTracker &t) {
            auto v = t.landmarks();
            py::array_t<float> a({(py::ssize_t)t.size(), (py::ssize_t)t.network().num_landmarks, (py::ssize_t)3});
            std::memcpy(a.mutable_data(), v.data(), v.size() * 4);
            return a;
        });

    // examples/facemesh.rs:35-56 on the device: track, detect on loss, re-seed from the best face
    py::class_<DeviceFaceLoop>(m, "DeviceFaceLoop")
        .def(py::init([](const std::string &detector, const std::string &landmarker, size_t streams, int device,
                         float padding, float loss, float det_threshold) {
                 return new DeviceFaceLoop(detector_net(detector), landmark_net(landmarker), streams, device, padding,
                                           loss, det_threshold);
             }), py::arg("detector") = "face", py::arg("landmarker") = "facemesh_v2", py::arg("streams") = 1,
             py::arg("device") = 0, py::arg("padding") = LandmarkTracker::DEFAULT_ROI_PADDING,
             py::arg("loss_threshold") = LandmarkTracker::DEFAULT_LOSS_THRESHOLD,
             py::arg("det_threshold") = Detector::DEFAULT_THRESHOLD)
        .def("set_roi", &DeviceFaceLoop::set_roi)
        .def("step", [](DeviceFaceLoop &t, const std::vector<std::tuple<uint64_t, uint32_t, uint32_t, uint64_t>> &frames) {
            std::vector<Image> im;
            for (auto &f : frames) {
                Image i;
                i.rgba = reinterpret_cast<const uint8_t *>(std::get<0>(f));
                i.width = std::get<1>(f);
                i.height = std::get<2>(f);
                i.row_stride = std::get<3>(f);
                i.on_device = true;
                im.push_back(i);
            }
            py::gil_scoped_release nogil;
            t.step(im);
        })
        .def("synchronize", &DeviceFaceLoop::synchronize, py::call_guard<py::gil_scoped_release>())
        .def("__len__", &DeviceFaceLoop::streams)
        .def("states", [](DeviceFaceLoop &t) {
            py::list out;
            for (const auto &s : t.states()) {
                py::dict d;
                d["roi"] = RotatedRect(Rect::from_center(s.roi[0], s.roi[1], s.roi[2], s.roi[3]), s.roi[4]);
                d["updated_roi"] = RotatedRect(Rect::from_center(s.updated[0], s.updated[1], s.updated[2], s.updated[3]), s.updated[4]);
                d["view_rect"] = RotatedRect(Rect::from_center(s.view_rect[0], s.view_rect[1], s.view_rect[2], s.view_rect[3]), s.view_rect[4]);
                d["active"] = s.active != 0;
                d["tracked"] = s.tracked != 0;
                d["confidence"] = s.confidence;
                out.append(d);
            }
            return out;
        })
        .def("landmarks", [](DeviceFaceLoop &t) {
            auto v = t.landmarks();
            py::array_t<float> a({(py::ssize_t)t.streams(), (py::ssize_t)t.landmarker().num_landmarks, (py::ssize_t)3});
            std::memcpy(a.mutable_data(), v.data(), v.size() * 4);
            return a;
        })
        .def("detected", &DeviceFaceLoop::detected)
        .def("detection_counts", &DeviceFaceLoop::detection_counts)
        .def("detections_run", &DeviceFaceLoop::detections_run)
        .def("reacquisitions", &DeviceFaceLoop::reacquisitions);

    py::class_<DetectTrackPipeline>(m, "DetectTrackPipeline")
        .def(py::init([](const std::string &kind, int device, int threads, uint32_t max_rois,
                         uint32_t sub_batches, bool stream_per_sub_batch, float loss_threshold,
                         const std::string &detector, const std::string &landmarker, bool device_post,
                         const std::string &nms_mode, uint32_t det_cap, float det_threshold) {
                 PipelineConfig c = kind == "hand" ? PipelineConfig::hand() : PipelineConfig::face();
                 if (kind != "hand" && kind != "face")
                     throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "pipeline kind must be 'face' or 'hand'");
                 // network overrides within a kind: BlazeFace full range / FaceMesh V2
                 //  run through the same pipeline as config 3
                 if (!detector.empty()) c.detector = detector_net(detector);
                 if (!landmarker.empty()) c.landmarker = landmark_net(landmarker);
                 c.max_rois_per_frame = max_rois;
                 c.sub_batches = sub_batches;
                 c.stream_per_sub_batch = stream_per_sub_batch;
                 c.loss_threshold = loss_threshold;  // LandmarkTracker::set_loss_threshold
                 c.device_post = device_post;
                 if (nms_mode == "remove") c.nms_mode = SuppressionMode::Remove;  // Detector::nms_mut
                 else if (nms_mode != "average") throw ZaruError(ZR_ERR_INVALID_ARGUMENT, "nms_mode: average | remove");
                 c.det_cap = det_cap;
                 c.det_threshold = det_threshold;  // Detector::set_threshold (detection.rs:191-193)
                 return new DetectTrackPipeline(c, device, threads);
             }), py::arg("kind") = "face", py::arg("device") = 0, py::arg("threads") = 8,
             py::arg("max_rois_per_frame") = 8, py::arg("sub_batches") = 2,
             py::arg("stream_per_sub_batch") = true,
             py::arg("loss_threshold") = LandmarkTracker::DEFAULT_LOSS_THRESHOLD,
             py::arg("detector") = "", py::arg("landmarker") = "", py::arg("device_post") = true,
             py::arg("nms_mode") = "average", py::arg("det_cap") = 0,
             py::arg("det_threshold") = Detector::DEFAULT_THRESHOLD)
        // frames: list of (device ptr, width, height, row_stride); forced: per frame list of
        // (cx, cy, w, h, rad) ROIs used when the frame has no detection
        .def("run", [](DetectTrackPipeline &p, const std::vector<std::tuple<uint64_t, uint32_t, uint32_t, uint64_t>> &frames,
                       const std::vector<std::vector<std::tuple<float, float, float, float, float>>> &forced) {
            std::vector<Image> im;
            for (auto &f : frames) {
                Image i;
                i.rgba = reinterpret_cast<const uint8_t *>(std::get<0>(f));
                i.width = std::get<1>(f);
                i.height = std::get<2>(f);
                i.row_stride = std::get<3>(f);
                i.on_device = true;
                im.push_back(i);
            }
            std::vector<std::vector<RotatedRect>> fr(forced.size());
            for (size_t k = 0; k < forced.size(); k++)
                for (auto &t : forced[k])
                    fr[k].push_back(RotatedRect(Rect::from_center(std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)), std::get<4>(t)));
            py::gil_scoped_release nogil;
            p.run(im, fr);
        })
        .def("set_frames", [](DetectTrackPipeline &p, const std::vector<std::tuple<uint64_t, uint32_t, uint32_t, uint64_t>> &frames,
                              const std::vector<std::vector<std::tuple<float, float, float, float, float>>> &forced) {
            std::vector<Image> im;
            for (auto &f : frames) {
                Image i;
                i.rgba = reinterpret_cast<const uint8_t *>(std::get<0>(f));
                i.width = std::get<1>(f);
                i.height = std::get<2>(f);
                i.row_stride = std::get<3>(f);
                i.on_device = true;
                im.push_back(i);
            }
            std::vector<std::vector<RotatedRect>> fr(forced.size());
            for (size_t k = 0; k < forced.size(); k++)
                for (auto &t : forced[k])
                    fr[k].push_back(RotatedRect(Rect::from_center(std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)), std::get<4>(t)));
            p.set_frames(std::move(im), std::move(fr));
        })
        .def("run_frames", [](DetectTrackPipeline &p) {
            py::gil_scoped_release nogil;
            p.run_frames();
            return p.rois().size();
        })
        .def("run_frames_repeated", [](DetectTrackPipeline &p, int steps) {
            py::gil_scoped_release nogil;
            p.run_frames_repeated(steps);
            return p.times().tracked;
        }, py::arg("steps"))
        .def("begin_steps", [](DetectTrackPipeline &p) {
            py::gil_scoped_release nogil;
            p.begin_steps();
        })
        .def("step", [](DetectTrackPipeline &p, bool more) {
            py::gil_scoped_release nogil;
            p.step(more);
            return p.times().tracked;
        }, py::arg("more"))
        .def("detections", [](const DetectTrackPipeline &p) { return p.detections(); })
        .def("detection_records", [](const DetectTrackPipeline &p, uint32_t rmax, uint32_t first_id,
                                     uint32_t id_stride) {
            const auto &d = p.detections();
            std::vector<uint32_t> ids(d.size());
            for (size_t i = 0; i < d.size(); i++) ids[i] = first_id + (uint32_t)i * id_stride;
            py::array_t<float> a({(py::ssize_t)d.size(), (py::ssize_t)det_record_width(rmax)});
            pack_detection_records(d, ids, rmax, a.mutable_data());
            return a;
        }, py::arg("rmax") = 8, py::arg("first_id") = 0, py::arg("id_stride") = 1)
        // device-written records, all-gathered over `comm` (a zaru_amd._lib.Comm
        // pointer, 0: none) on the pipeline's own stream
        .def("enable_records", [](DetectTrackPipeline &p, uint32_t rmax, uint32_t first_id, uint32_t id_stride,
                                  uint64_t comm, int world) {
            p.enable_records(rmax, first_id, id_stride, reinterpret_cast<zr_comm *>(comm), world);
        }, py::arg("rmax") = 8, py::arg("first_id") = 0, py::arg("id_stride") = 1, py::arg("comm") = 0,
           py::arg("world") = 1)
        .def("records", [](DetectTrackPipeline &p) {
            std::vector<float> r;
            {
                py::gil_scoped_release nogil;
                r = p.records();
            }
            const py::ssize_t w = p.record_width();
            py::array_t<float> a({(py::ssize_t)r.size() / w, w});
            std::memcpy(a.mutable_data(), r.data(), r.size() * 4);
            return a;
        })
        .def("gathered", [](DetectTrackPipeline &p) {
            std::vector<float> r;
            {
                py::gil_scoped_release nogil;
                r = p.gathered();
            }
            const py::ssize_t w = p.record_width();
            py::array_t<float> a({(py::ssize_t)r.size() / w, w});
            std::memcpy(a.mutable_data(), r.data(), r.size() * 4);
            return a;
        })
        .def("num_rois", [](const DetectTrackPipeline &p) { return p.rois().size(); })
        .def("roi", [](const DetectTrackPipeline &p, size_t i) {
            const RoiResult &r = p.rois().at(i);
            py::dict d = estimate_dict(r.result.estimate);
            d["frame"] = r.frame;
            d["from_detection"] = r.from_detection;
            d["tracked"] = r.tracked;
            d["confidence"] = r.confidence;
            d["roi"] = r.roi;
            d["view_rect"] = r.result.view_rect;
            d["updated_roi"] = r.result.updated_roi;
            d["next_roi"] = r.next_roi;
            return d;
        })
        .def("times", [](const DetectTrackPipeline &p) {
            const StageTimes &t = p.times();
            py::dict d;
            d["detect_gpu_ms"] = t.detect_gpu_ms;
            d["decode_nms_ms"] = t.decode_nms_ms;
            d["landmark_gpu_ms"] = t.landmark_gpu_ms;
            d["map_ms"] = t.map_ms;
            d["total_ms"] = t.total_ms;
            d["host_wait_ms"] = t.host_wait_ms;
            d["dropped_detections"] = t.dropped_detections;
            d["nms_candidates"] = t.nms_candidates;
            d["nms_tied"] = t.nms_tied;
            d["nms_unpinned_frames"] = t.nms_unpinned_frames;
            d["frames"] = t.frames;
            d["detections"] = t.detections;
            d["rois"] = t.rois;
            d["tracked"] = t.tracked;
            return d;
        })
        .def("stats", [](const DetectTrackPipeline &p) {
            py::dict d;
            d["detector_bytes_per_image"] = p.detector_bytes_per_image();
            d["landmarker_bytes_per_image"] = p.landmarker_bytes_per_image();
            d["detector_flops_per_image"] = p.detector_flops_per_image();
            d["landmarker_flops_per_image"] = p.landmarker_flops_per_image();
            return d;
        })
        .def("stream", [](const DetectTrackPipeline &p) { return reinterpret_cast<uint64_t>(p.stream()); })
        .def("profile", &DetectTrackPipeline::profile)
        .def("profile_read", &DetectTrackPipeline::profile_read);
}
