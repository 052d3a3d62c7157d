// Robot model: host-side URDF/SRDF build and the flat device image the
// kernels read.  Restates Pinocchio's model/geometry build as the reference
// uses it in Manipulator::RobotData::RobotData (src/manipulator/robot_data.cpp:7-70).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace drc_amd {

constexpr int kMaxJoints = 16;    // 1-DoF joints (XLS-FR3 needs 14)
constexpr int kMaxGeoms = 64;
constexpr int kMaxPairs = 1024;
constexpr int kMaxFrames = 64;
constexpr int kMaxWheels = 8;
constexpr int kMaxCandSlots = 128;  // non-sphere pairs the lane-per-instance task stage tracks

enum JointType : int { kRevolute = 0, kPrismatic = 1 };
enum GeomType : int { kSphere = 0, kCylinder = 1, kBox = 2 };
enum DriveKind : int { kDriveDifferential = 0, kDriveMecanum = 1, kDriveCaster = 2 };  // DRC_DRIVE_*

// Flat, POD model image in HBM.  Transforms are 12 doubles: R row-major, p.
struct DevModel {
  int nv, ngeom, npairs, nframes;
  int kind;                        // 0 manipulator, 1 mobile manipulator
  int n_arm, n_wheel;
  int virtual_start, mani_start, mobi_start;
  int act_mani_start, act_mobi_start;
  int parent[kMaxJoints + 1];
  int jtype[kMaxJoints + 1];
  uint32_t anc[kMaxJoints + 1];    // bit (k-1) set iff joint k supports joint j (inclusive)
  double jplace[kMaxJoints + 1][12];
  double axis[kMaxJoints + 1][3];
  double lower[kMaxJoints], upper[kMaxJoints], vel[kMaxJoints];
  int frame_joint[kMaxFrames];
  double frame_place[kMaxFrames][12];
  int gparent[kMaxGeoms];
  int gtype[kMaxGeoms];
  double gplace[kMaxGeoms][12];
  double gparam[kMaxGeoms][3];     // sphere r | cylinder r, h/2 | box half extents
  double gbound[kMaxGeoms];        // conservative core/bounding radius for the broad phase
  int16_t pair_a[kMaxPairs], pair_b[kMaxPairs];
  int16_t cand_slot[kMaxPairs];       // pair -> GJK candidate slot (pairs without a sphere), or -1
  int16_t cand_pair[kMaxCandSlots];   // slot -> pair
  int ncand_slots;                    // non-sphere pairs (> kMaxCandSlots: lane stage not used)
  int16_t pair_order[kMaxPairs];      // pairs grouped by shape-type class (pair index order within a class):
                                      // the wave kernel's lanes then take same-type pairs in each round
  int16_t slot_a[kMaxPairs], slot_b[kMaxPairs];  // pair_a / pair_b of pair_order[slot]: one load level less
  double J_mobile[3][kMaxWheels];  // base twist = J_mobile * wheel velocity (differential, mecanum)
  int drive;                       // DriveKind; caster: J_mobile depends on the steer angles (mobile_fk.hpp)
  double wheel_radius, wheel_offset;
  double caster_pos[kMaxWheels / 2][2];  // base2wheel_positions of the casters
  // rigid-body inertia carried by each joint (links behind fixed joints merged,
  // Pinocchio appendBodyToJoint), in the joint frame:
  // {mass, com x, y, z, Ixx, Iyy, Izz, Ixy, Ixz, Iyz} with I about the com
  double inertia[kMaxJoints + 1][10];
  int dyn_origin;                  // joint whose origin the dynamics kernel takes as spatial reference (0 = world)
};

struct HostModel {
  DevModel dev{};
  std::vector<std::string> joint_names;   // index j-1
  std::vector<std::string> frame_names;   // link (BODY) frames, index = frame id
  std::vector<std::string> geom_names;
  std::vector<double> effort;
};

// Returns 0 on success, DRC_ERR_* otherwise; err gets a readable reason.
int build_model_from_urdf(const std::string& urdf_path, const std::string& srdf_path,
                          HostModel* out, std::string* err);

}  // namespace drc_amd
