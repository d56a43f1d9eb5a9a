/* lvp_layout_probe.c -- test infrastructure (a checker, never linked into the product).
 *
 * Prints, as JSON, the byte layout of the lavapipe / Vulkan structures that the driver-side drop-in
 * (tests/integration/vksim_shim.cpp) reads through its layout mirror. The numbers come from the reference's own
 * definitions, compiled where they lie under /root/reference by oracle/Makefile (target lvp-layout):
 *   - mesa-vulkan-sim/include/vulkan/vulkan_core.h            (VkAccelerationStructureGeometryKHR, instances,
 *                                                              VkRayTracingPipelineCreateInfoKHR, ...)
 *   - mesa-vulkan-sim/src/gallium/include/pipe/p_state.h      (pipe_shader_buffer / pipe_constant_buffer /
 *                                                              pipe_image_view: the fork's pmem / image fields)
 *   - mesa-vulkan-sim/src/vulkan/runtime/vk_object.h, vk_descriptor_set_layout.h, vk_image.h
 *   - mesa-vulkan-sim/src/gallium/frontends/lavapipe/lvp_private.h:257-265 (lvp_image) and :284-371
 *     (lvp_descriptor_set_binding_layout, lvp_descriptor_set_layout, lvp_descriptor, lvp_descriptor_set).
 *     lvp_private.h as a whole needs generated headers (lvp_entrypoints.h) that only a meson build makes, so the
 *     Makefile compiles those line ranges of it, unmodified, after the real headers they depend on.
 * tests/golden/make_lvp_layout.py runs this and commits the output as tests/golden/lvp_layout.json.
 */
#include <stddef.h>
#include <stdio.h>

#include "pipe/p_state.h"
#include "util/list.h"
#include "vk_descriptor_set_layout.h"
#include "vk_image.h"
#include "vk_object.h"

#define LVP_SHADER_STAGES MESA_ALL_SHADER_STAGES           /* lvp_private.h:118 */
#define MAX_PER_STAGE_DESCRIPTOR_UNIFORM_BLOCKS 8          /* lvp_private.h:88 */
#include "lvp_slice_image.h"
#include "lvp_slice_descriptors.h"

#define F(T, f) printf("  \"%s.%s\": %zu,\n", #T, #f, offsetof(T, f))
#define S(T) printf("  \"sizeof %s\": %zu,\n", #T, sizeof(T))

int main(void) {
    printf("{\n");
    /* lavapipe descriptor set (lvp_private.h:284-371) */
    S(struct lvp_descriptor_set);
    F(struct lvp_descriptor_set, layout);
    F(struct lvp_descriptor_set, descriptors);
    S(struct lvp_descriptor);
    F(struct lvp_descriptor, type);
    F(struct lvp_descriptor, info);
    F(struct lvp_descriptor, info.ssbo.pmem);
    F(struct lvp_descriptor, info.ssbo.buffer_offset);
    F(struct lvp_descriptor, info.ssbo.buffer_size);
    F(struct lvp_descriptor, info.ubo.pmem);
    F(struct lvp_descriptor, info.ubo.buffer_offset);
    F(struct lvp_descriptor, info.ubo.buffer_size);
    F(struct lvp_descriptor, info.image_view.image);
    F(struct lvp_descriptor_set_layout, binding_count);
    F(struct lvp_descriptor_set_layout, binding);
    S(struct lvp_descriptor_set_binding_layout);
    F(struct lvp_descriptor_set_binding_layout, descriptor_index);
    F(struct lvp_descriptor_set_binding_layout, type);
    F(struct lvp_descriptor_set_binding_layout, array_size);
    /* lvp_image (lvp_private.h:257-265) and its vk_image prefix */
    F(struct lvp_image, vk.format);
    F(struct lvp_image, vk.extent);
    F(struct lvp_image, vk.tiling);
    /* Vulkan API structures the driver hands to the simulator */
    S(VkAccelerationStructureGeometryKHR);
    F(VkAccelerationStructureGeometryKHR, geometryType);
    F(VkAccelerationStructureGeometryKHR, geometry);
    F(VkAccelerationStructureGeometryKHR, flags);
    F(VkAccelerationStructureGeometryTrianglesDataKHR, vertexFormat);
    F(VkAccelerationStructureGeometryTrianglesDataKHR, vertexData);
    F(VkAccelerationStructureGeometryTrianglesDataKHR, vertexStride);
    F(VkAccelerationStructureGeometryTrianglesDataKHR, maxVertex);
    F(VkAccelerationStructureGeometryTrianglesDataKHR, indexType);
    F(VkAccelerationStructureGeometryTrianglesDataKHR, indexData);
    F(VkAccelerationStructureGeometryAabbsDataKHR, data);
    F(VkAccelerationStructureGeometryAabbsDataKHR, stride);
    F(VkAccelerationStructureGeometryInstancesDataKHR, arrayOfPointers);
    F(VkAccelerationStructureGeometryInstancesDataKHR, data);
    S(VkAccelerationStructureInstanceKHR);
    F(VkAccelerationStructureInstanceKHR, accelerationStructureReference);
    S(VkRayTracingPipelineCreateInfoKHR);
    F(VkRayTracingPipelineCreateInfoKHR, stageCount);
    F(VkRayTracingPipelineCreateInfoKHR, pStages);
    F(VkRayTracingPipelineCreateInfoKHR, groupCount);
    F(VkRayTracingPipelineCreateInfoKHR, pGroups);
    S(VkRayTracingShaderGroupCreateInfoKHR);
    F(VkRayTracingShaderGroupCreateInfoKHR, type);
    F(VkRayTracingShaderGroupCreateInfoKHR, generalShader);
    F(VkRayTracingShaderGroupCreateInfoKHR, closestHitShader);
    F(VkRayTracingShaderGroupCreateInfoKHR, anyHitShader);
    F(VkRayTracingShaderGroupCreateInfoKHR, intersectionShader);
    S(VkPipelineShaderStageCreateInfo);
    F(VkPipelineShaderStageCreateInfo, stage);
    /* enum values the shim tests */
    printf("  \"VK_GEOMETRY_TYPE_TRIANGLES_KHR\": %d,\n", (int)VK_GEOMETRY_TYPE_TRIANGLES_KHR);
    printf("  \"VK_GEOMETRY_TYPE_AABBS_KHR\": %d,\n", (int)VK_GEOMETRY_TYPE_AABBS_KHR);
    printf("  \"VK_GEOMETRY_TYPE_INSTANCES_KHR\": %d,\n", (int)VK_GEOMETRY_TYPE_INSTANCES_KHR);
    printf("  \"VK_DESCRIPTOR_TYPE_STORAGE_IMAGE\": %d,\n", (int)VK_DESCRIPTOR_TYPE_STORAGE_IMAGE);
    printf("  \"VK_DESCRIPTOR_TYPE_UNIFORM_BUFFER\": %d,\n", (int)VK_DESCRIPTOR_TYPE_UNIFORM_BUFFER);
    printf("  \"VK_DESCRIPTOR_TYPE_STORAGE_BUFFER\": %d,\n", (int)VK_DESCRIPTOR_TYPE_STORAGE_BUFFER);
    printf("  \"VK_DESCRIPTOR_TYPE_ACCELERATION_STRUCTURE_KHR\": %d,\n",
           (int)VK_DESCRIPTOR_TYPE_ACCELERATION_STRUCTURE_KHR);
    printf("  \"VK_RAY_TRACING_SHADER_GROUP_TYPE_GENERAL_KHR\": %d,\n", (int)VK_RAY_TRACING_SHADER_GROUP_TYPE_GENERAL_KHR);
    printf("  \"VK_RAY_TRACING_SHADER_GROUP_TYPE_TRIANGLES_HIT_GROUP_KHR\": %d,\n",
           (int)VK_RAY_TRACING_SHADER_GROUP_TYPE_TRIANGLES_HIT_GROUP_KHR);
    printf("  \"VK_RAY_TRACING_SHADER_GROUP_TYPE_PROCEDURAL_HIT_GROUP_KHR\": %d,\n",
           (int)VK_RAY_TRACING_SHADER_GROUP_TYPE_PROCEDURAL_HIT_GROUP_KHR);
    printf("  \"VK_SHADER_STAGE_INTERSECTION_BIT_KHR\": %d,\n", (int)VK_SHADER_STAGE_INTERSECTION_BIT_KHR);
    printf("  \"VK_FORMAT_R32G32B32_SFLOAT\": %d,\n", (int)VK_FORMAT_R32G32B32_SFLOAT);
    printf("  \"VK_FORMAT_R32G32B32A32_SFLOAT\": %d,\n", (int)VK_FORMAT_R32G32B32A32_SFLOAT);
    printf("  \"VK_FORMAT_B8G8R8A8_UNORM\": %d,\n", (int)VK_FORMAT_B8G8R8A8_UNORM);
    printf("  \"VK_INDEX_TYPE_UINT32\": %d,\n", (int)VK_INDEX_TYPE_UINT32);
    printf("  \"MESA_SHADER_RAYGEN\": %d,\n", (int)MESA_SHADER_RAYGEN);
    printf("  \"MESA_SHADER_INTERSECTION\": %d\n", (int)MESA_SHADER_INTERSECTION);
    printf("}\n");
    return 0;
}
