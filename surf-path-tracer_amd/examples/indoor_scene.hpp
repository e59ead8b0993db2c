/*
 * indoor_scene.hpp -- the reference application's scene (sources/main.cpp:
 * 141-149 camera, :161-346 meshes, BLASes, materials, instances, background)
 * built with the drop-in C++ API, shared by the examples.  The objects live in
 * one struct because Instance / GPUScene keep pointers to them, as the
 * reference's main() keeps them on its stack.
 */
#pragma once
#include "surf/surf_host.hpp"

#include <memory>
#include <string>
#include <vector>

namespace surf {

struct IndoorScene {
    Mesh susanneMesh, cubeMesh, lensMesh, planeMesh;
    BvhBLAS susanneBlas, cubeBlas, lensBlas, planeBlas;
    Material floorMat, wallRed, wallGreen, diffuseMat, dielectricMat, specularMat, softLight, redLight;
    std::unique_ptr<GPUScene> scene;

    IndoorScene(RenderContext* context, const std::string& dir)
        : susanneMesh(dir + "/susanne.obj"), cubeMesh(dir + "/cube.obj"), lensMesh(dir + "/lens.obj"), planeMesh(dir + "/plane.obj"),
          susanneBlas(&susanneMesh), cubeBlas(&cubeMesh), lensBlas(&lensMesh), planeBlas(&planeMesh) {
        floorMat.albedo = Float3(0.8f); floorMat.reflectivity = 0.01f;
        wallRed.albedo = Float3(1.0f, 0.0f, 0.0f);
        wallGreen.albedo = Float3(0.0f, 1.0f, 0.0f);
        diffuseMat.albedo = Float3(1.0f, 0.0f, 0.0f);
        dielectricMat.albedo = Float3(0.7f, 0.7f, 0.2f); dielectricMat.absorption = Float3(0.03f, 0.04f, 0.03f);
        dielectricMat.refractivity = 1.0f; dielectricMat.indexOfRefraction = 1.42f;
        specularMat.albedo = Float3(0.2f, 0.9f, 1.0f); specularMat.reflectivity = 0.8f;
        softLight.emissionColor = Float3(1.0f, 0.8f, 0.6f); softLight.emissionStrength = 5.0f;
        redLight.emissionColor = Float3(1.0f, 0.5f, 0.2f); redLight.emissionStrength = 5.0f;

        const Mat4 I(1.0f);
        std::vector<Instance> instances;
        instances.emplace_back(&planeBlas, &floorMat, scale(translate(I, Float3(0.0f, -1.0f, 0.0f)), Float3(10.0f, 10.0f, 10.0f)));
        instances.emplace_back(&cubeBlas, &softLight, scale(translate(I, Float3(-8.0f, 7.0f, 5.0f)), Float3(0.5f, 0.5f, 0.5f)));
        instances.emplace_back(&cubeBlas, &redLight, scale(translate(I, Float3(9.0f, 5.0f, -5.0f)), Float3(1.0f, 1.0f, 1.0f)));
        instances.emplace_back(&susanneBlas, &diffuseMat, translate(I, Float3(0.0f, 0.0f, -1.0f)));
        instances.emplace_back(&susanneBlas, &specularMat, translate(I, Float3(3.0f, 0.0f, -1.0f)));
        instances.emplace_back(&lensBlas, &dielectricMat, translate(I, Float3(-3.0f, 0.0f, -1.0f)));
        instances.emplace_back(&planeBlas, &wallRed, scale(rotate(translate(I, Float3(-10.0f, 4.0f, 0.0f)), radians(90.0f), WORLD_FORWARD), Float3(5.0f, 10.0f, 10.0f)));
        instances.emplace_back(&planeBlas, &wallGreen, scale(rotate(translate(I, Float3(10.0f, 4.0f, 0.0f)), radians(90.0f), WORLD_FORWARD), Float3(5.0f, 10.0f, 10.0f)));
        instances.emplace_back(&planeBlas, &floorMat, scale(translate(I, Float3(0.0f, 9.0f, 0.0f)), Float3(10.0f, 10.0f, 10.0f)));
        instances.emplace_back(&planeBlas, &floorMat, scale(rotate(translate(I, Float3(0.0f, 4.0f, -10.0f)), radians(90.0f), WORLD_RIGHT), Float3(10.0f, 10.0f, 5.0f)));
        instances.emplace_back(&planeBlas, &floorMat, scale(rotate(translate(I, Float3(0.0f, 4.0f, 10.0f)), radians(90.0f), WORLD_RIGHT), Float3(10.0f, 10.0f, 5.0f)));

        SceneBackground background;
        background.type = BackgroundType::ColorGradient;
        background.gradient.colorA = Float3(0.8f, 0.8f, 0.8f);
        background.gradient.colorB = Float3(0.1f, 0.4f, 0.6f);
        scene = std::make_unique<GPUScene>(context, background, instances);
    }
    IndoorScene(const IndoorScene&) = delete;
    IndoorScene& operator=(const IndoorScene&) = delete;
};

/* main.cpp:141-149: position (0,0,-7) looking at the origin, fov 70, focal 7, defocus 0.5. */
inline Camera indoorCamera(U32 width, U32 height) {
    return Camera(Float3(0.0f, 0.0f, -7.0f), Float3(0.0f, 0.0f, 0.0f), width, height, 70.0f, 7.0f, 0.5f);
}

}  // namespace surf
